// Microbenchmark (diagnostic, not shipped): ways to gather 16 bytes from a byte-unaligned LDS
// offset, lane c reading [16 c + d, 16 c + d + 16) (d per lane-segment, as the decode's copy
// windows do). 256 workgroups x 1024 threads, each lane ITERS gathers; prints ms per variant and
// checks every variant's bytes against the reference gather.
//   0 b64x3 : three 8-byte-aligned ds_read_b64 + dword selects + alignbyte (the shipped gather)
//   1 u64x2 : two ds_read_b64 at the byte address (unaligned)
//   2 u32x4 : four ds_read_b32 at the byte address (unaligned)
//   3 u128  : one ds_read_b128 at the byte address (unaligned)
//   4 glob  : one global_load_dwordx4 at the byte address (an L2-resident buffer)
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr int ITERS = 2048;
constexpr int kWin = 4352;
typedef uint32_t u32;
typedef u32 u32x2 __attribute__((ext_vector_type(2)));
typedef u32 u32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(1024, 4) void k(u32* out, const uint8_t* gsrc, u32 seed) {
  __shared__ __attribute__((aligned(16))) uint8_t win[16 * kWin + 64];
  for (int i = threadIdx.x; i < 16 * kWin / 4; i += 1024)
    reinterpret_cast<u32*>(win)[i] = (u32)(i % (kWin / 4)) * 2654435761u ^ 0x5bd1e995u;
  __syncthreads();
  const u32 lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint8_t* w = win + wv * kWin;
  const uint8_t* g = gsrc + (blockIdx.x & 63) * kWin;
  u32 x = seed ^ (threadIdx.x * 0x9E3779B9u);
  u32 acc = 0;
  for (int it = 0; it < ITERS; it++) {
    const u32 d = (x >> 8) & 127;           // segment delta (same for 8-lane runs)
    const int off = (int)((16 * (lane & 63)) % 4096 + ((d + (lane >> 3)) & 127)) & ~0 ;
    const int o = off < kWin - 24 ? off : off - 128;
    u32x4 v;
    if (MODE == 0) {
      const u32x2* p = reinterpret_cast<const u32x2*>(w + (o & ~7));
      const u32x2 a = p[0], b = p[1], c = p[2];
      const u32 s = o & 3u;
      const u32 sel = (o & 4) ? 0x07060504u : 0x03020100u;
      const u32 s0 = __builtin_amdgcn_perm(a.y, a.x, sel), s1 = __builtin_amdgcn_perm(b.x, a.y, sel),
                s2 = __builtin_amdgcn_perm(b.y, b.x, sel), s3 = __builtin_amdgcn_perm(c.x, b.y, sel),
                s4 = __builtin_amdgcn_perm(c.y, c.x, sel);
      v = u32x4{__builtin_amdgcn_alignbyte(s1, s0, s), __builtin_amdgcn_alignbyte(s2, s1, s),
                __builtin_amdgcn_alignbyte(s3, s2, s), __builtin_amdgcn_alignbyte(s4, s3, s)};
    } else if (MODE == 1) {   // (inline asm: the compiler merges unaligned reads into b128)
      const u32 la = (u32)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)(w + o);
      u32x2 a, b;
      asm volatile("ds_read_b64 %0, %2\n\tds_read_b64 %1, %2 offset:8\n\ts_waitcnt lgkmcnt(0)"
                   : "=v"(a), "=v"(b) : "v"(la));
      v = u32x4{a.x, a.y, b.x, b.y};
    } else if (MODE == 2) {
      const u32 la = (u32)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)(w + o);
      u32 p0, p1, p2, p3;
      asm volatile("ds_read_b32 %0, %4\n\tds_read_b32 %1, %4 offset:4\n\tds_read_b32 %2, %4 offset:8\n\t"
                   "ds_read_b32 %3, %4 offset:12\n\ts_waitcnt lgkmcnt(0)"
                   : "=v"(p0), "=v"(p1), "=v"(p2), "=v"(p3) : "v"(la));
      v = u32x4{p0, p1, p2, p3};
    } else if (MODE == 3) {
      typedef u32x4 u32x4u __attribute__((aligned(1)));
      v = *reinterpret_cast<const u32x4u*>(w + o);
    } else {
      typedef u32x4 u32x4u __attribute__((aligned(1)));
      v = *reinterpret_cast<const u32x4u*>(g + o);
    }
    const u32 c = v.x ^ v.y ^ v.z ^ v.w;
    x = x * 1664525u + 1013904223u;   // independent gathers: a throughput test
    acc += c;
  }
  out[blockIdx.x * 1024 + threadIdx.x] = acc;
}

template <int M>
float run(u32* d, const uint8_t* g) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  k<M><<<256, 1024>>>(d, g, 1);
  hipDeviceSynchronize();
  hipEventRecord(a);
  k<M><<<256, 1024>>>(d, g, 2);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  u32* d;
  uint8_t* g;
  hipMalloc(&d, 256 * 1024 * 4 * 5);
  hipMalloc(&g, 64 * kWin + 64);
  // the global buffer holds the same bytes as every wave's LDS window (for the check)
  u32* h = new u32[kWin / 4];
  for (int i = 0; i < kWin / 4; i++) h[i] = (u32)i * 2654435761u ^ 0x5bd1e995u;
  for (int b = 0; b < 64; b++) hipMemcpy(g + b * kWin, h, kWin, hipMemcpyHostToDevice);
  const char* names[] = {"b64x3+perm+align", "u64x2 unaligned", "u32x4 unaligned", "u128 unaligned",
                         "global dwordx4 unaligned"};
  float ms[5] = {run<0>(d, g), run<1>(d + 256 * 1024, g), run<2>(d + 2 * 256 * 1024, g),
                 run<3>(d + 3 * 256 * 1024, g), run<4>(d + 4 * 256 * 1024, g)};
  u32* o = new u32[256 * 1024 * 5];
  hipMemcpy(o, d, 256 * 1024 * 4 * 5, hipMemcpyDeviceToHost);
  for (int m = 0; m < 5; m++) {
    // wave 0 of workgroup 0 reads the same window bytes as the global copy (workgroup 0)
    int bad = 0;
    for (int t = 0; t < 64; t++) bad += o[m * 256 * 1024 + t] != o[t];
    printf("{\"variant\": \"%s\", \"ms\": %.4f, \"ns_per_gather_per_cu\": %.3f, \"mismatch_lanes\": %d}\n",
           names[m], ms[m], ms[m] * 1e6 / (16.0 * 64 * ITERS), bad);
  }
  return 0;
}
