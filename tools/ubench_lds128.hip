// Microbenchmark (diagnostic, not shipped): 16-byte LDS reads at arbitrary byte offsets on gfx950.
// Compares one unaligned ds_read_b128 with two aligned ds_read_b128 + funnel shift, checks that
// the unaligned read returns the right bytes, and times each pattern.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef uint32_t u32;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_a1 __attribute__((aligned(1)));
constexpr int ITERS = 2048, LDSB = 8192;

__device__ __forceinline__ u32x4 funnel(const uint8_t* base, int x) {
  const u32x4* p = reinterpret_cast<const u32x4*>(base + (x & ~15));
  u32x4 a = p[0], b = p[1];
  asm volatile("" : "+v"(a), "+v"(b));
  const u32 sh = (u32)x & 15u, s = sh & 3u, q = sh >> 2;
  const u32 w0 = q < 2 ? (q == 0 ? a.x : a.y) : (q == 2 ? a.z : a.w);
  const u32 w1 = q < 2 ? (q == 0 ? a.y : a.z) : (q == 2 ? a.w : b.x);
  const u32 w2 = q < 2 ? (q == 0 ? a.z : a.w) : (q == 2 ? b.x : b.y);
  const u32 w3 = q < 2 ? (q == 0 ? a.w : b.x) : (q == 2 ? b.y : b.z);
  const u32 w4 = q < 2 ? (q == 0 ? b.x : b.y) : (q == 2 ? b.z : b.w);
  u32x4 r;
  r.x = __builtin_amdgcn_alignbyte(w1, w0, s); r.y = __builtin_amdgcn_alignbyte(w2, w1, s);
  r.z = __builtin_amdgcn_alignbyte(w3, w2, s); r.w = __builtin_amdgcn_alignbyte(w4, w3, s);
  return r;
}

// MODE 0: aligned b128, lane-contiguous; 1: unaligned b128, lane stride 16 + per-lane offset
// (0..15); 2: funnel (2 aligned b128 + selects); 3: unaligned b128, lane stride 20 (entry-like);
// 4: dword-aligned b128 (offset multiple of 4)
template <int MODE>
__global__ __launch_bounds__(1024, 4) void k(u32* out, u32 seed) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[16][LDSB];
  const u32 w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int i = lane; i < LDSB; i += 64) lds[w][i] = (uint8_t)(i * 7 + w);
  __syncthreads();
  u32 x = seed ^ (threadIdx.x * 0x9E3779B9u);
  u32 acc = 0;
  for (int it = 0; it < ITERS; it++) {
    const u32 jit = (x >> 7) & 15u;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      u32x4 v;
      const int o = j * 1024;
      if (MODE == 0) v = *reinterpret_cast<const u32x4*>(&lds[w][(o + lane * 16) & (LDSB - 1)]);
      if (MODE == 1) v = *reinterpret_cast<const u32x4_a1*>(&lds[w][(o + lane * 16 + jit) & (LDSB - 32)] + jit);
      if (MODE == 2) v = funnel(lds[w], ((o + lane * 16) & (LDSB - 32)) + jit);
      if (MODE == 3) v = *reinterpret_cast<const u32x4_a1*>(&lds[w][((o + lane * 20) & (LDSB - 64)) + jit]);
      if (MODE == 4) v = *reinterpret_cast<const u32x4_a1*>(&lds[w][((o + lane * 16) & (LDSB - 32)) + (jit & 12)]);
      acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    x = x * 1664525u + 1013904223u + (acc & 1);
  }
  out[blockIdx.x * 1024 + threadIdx.x] = acc;
}

__global__ void check(u32* bad) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[512];
  for (int i = threadIdx.x; i < 512; i += 64) lds[i] = (uint8_t)(i * 13 + 5);
  __syncthreads();
  for (int x = threadIdx.x; x < 480; x += 64) {
    const u32x4 v = *reinterpret_cast<const u32x4_a1*>(lds + x);
    const u32x4 f = funnel(lds, x);
    u32 e[4] = {0, 0, 0, 0};
    for (int k = 0; k < 16; k++) e[k >> 2] |= (u32)(uint8_t)((x + k) * 13 + 5) << (8 * (k & 3));
    if (v.x != e[0] || v.y != e[1] || v.z != e[2] || v.w != e[3]) atomicAdd(bad, 1u);
    if (f.x != e[0] || f.y != e[1] || f.z != e[2] || f.w != e[3]) atomicAdd(bad + 1, 1u);
  }
}

template <int M> float run(u32* d) {
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  k<M><<<256, 1024>>>(d, 1); (void)hipDeviceSynchronize();
  (void)hipEventRecord(a); k<M><<<256, 1024>>>(d, 2); (void)hipEventRecord(b); (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b); return ms;
}
int main() {
  u32* d; (void)hipMalloc(&d, 256 * 1024 * 4);
  u32* bad; (void)hipMalloc(&bad, 8); (void)hipMemset(bad, 0, 8);
  check<<<1, 64>>>(bad);
  u32 hb[2]; (void)hipMemcpy(hb, bad, 8, hipMemcpyDeviceToHost);
  printf("unaligned ds_read_b128 mismatches: %u, funnel mismatches: %u\n", hb[0], hb[1]);
  const char* names[] = {"aligned b128", "unaligned b128 (stride16+j)", "funnel 2xb128+select",
                         "unaligned b128 (stride20)", "dword-aligned b128"};
  float ms[5] = {run<0>(d), run<1>(d), run<2>(d), run<3>(d), run<4>(d)};
  for (int m = 0; m < 5; m++) {
    double instr_per_cu = 16.0 * ITERS * 8;  // 16 waves/CU x ITERS x 8 reads
    printf("%-32s %8.3f ms  %6.2f cyc@2.4GHz per wave-read per CU\n", names[m], ms[m],
           ms[m] * 1e6 / instr_per_cu * 2.4);
  }
  return 0;
}
