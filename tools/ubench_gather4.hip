// Microbenchmark (diagnostic, not shipped): 16-byte gathers from byte-unaligned LDS offsets built
// from 4-byte-aligned reads (5 dwords + 4 v_alignbyte, no dword selects), against the shipped
// gather (three 8-byte-aligned ds_read_b64 + 5 selects + 4 alignbyte). Same access pattern as
// tools/ubench_gather.hip: lane c reads [16 c + d, 16 c + d + 16), d shared by 8-lane runs.
//   0 ship   : three 8-aligned ds_read_b64 + 5 v_cndmask + 4 v_alignbyte (lds_window16)
//   1 b128a4 : ds_read_b128 at the 4-aligned address + ds_read_b32 at +16 + 4 v_alignbyte
//   2 b64a4  : two ds_read_b64 at the 4-aligned address (+0, +8) + ds_read_b32 at +16 + 4 align
//   3 r2b32  : ds_read2_b32 (+0, +4) + ds_read2_b32 (+8, +12) + ds_read_b32 (+16) + 4 align
//   4 b96a4  : ds_read_b96 at the 4-aligned address + ds_read_b64 at +12 + 4 align
// 256 workgroups x 1024 threads; prints ms per variant and whether its bytes equal mode 0's.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr int ITERS = 2048;
constexpr int kWin = 4352;
typedef uint32_t u32;
typedef u32 u32x2 __attribute__((ext_vector_type(2)));
typedef u32 u32x3 __attribute__((ext_vector_type(3)));
typedef u32 u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32 lds_addr(const uint8_t* p) {
  return (u32)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)p;
}

template <int MODE>
__global__ __launch_bounds__(1024, 4) void k(u32* out, u32 seed) {
  __shared__ __attribute__((aligned(16))) uint8_t win[16 * kWin + 64];
  for (int i = threadIdx.x; i < 16 * kWin / 4; i += 1024)
    reinterpret_cast<u32*>(win)[i] = (u32)(i % (kWin / 4)) * 2654435761u ^ 0x5bd1e995u;
  __syncthreads();
  const u32 lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint8_t* w = win + wv * kWin;
  u32 x = seed ^ (threadIdx.x * 0x9E3779B9u);
  u32 acc = 0, first = 0;
  for (int it = 0; it < ITERS; it++) {
    const u32 d = (x >> 8) & 127;
    const int off = (int)((16 * (lane & 63)) % 4096 + ((d + (lane >> 3)) & 127));
    const int o = off < kWin - 24 ? off : off - 128;
    u32x4 v;
    if (MODE == 0) {
      const u32x2* p = reinterpret_cast<const u32x2*>(w + (o & ~7));
      u32x2 a = p[0], b = p[1], c = p[2];
      asm volatile("" : "+v"(a), "+v"(b), "+v"(c));
      const u32 s = (u32)o & 3u;
      const bool h = ((u32)o & 4u) != 0;
      const u32 s0 = h ? a.y : a.x, s1 = h ? b.x : a.y, s2 = h ? b.y : b.x, s3 = h ? c.x : b.y,
                s4 = h ? c.y : c.x;
      v = u32x4{__builtin_amdgcn_alignbyte(s1, s0, s), __builtin_amdgcn_alignbyte(s2, s1, s),
                __builtin_amdgcn_alignbyte(s3, s2, s), __builtin_amdgcn_alignbyte(s4, s3, s)};
    } else {
      const u32 la = lds_addr(w + (o & ~3));
      u32 q0, q1, q2, q3, q4;
      if (MODE == 1) {
        u32x4 a;
        u32 b;
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b32 %1, %2 offset:16\n\ts_waitcnt lgkmcnt(0)"
                     : "=v"(a), "=v"(b) : "v"(la));
        q0 = a.x, q1 = a.y, q2 = a.z, q3 = a.w, q4 = b;
      } else if (MODE == 2) {
        u32x2 a, b;
        u32 c;
        asm volatile("ds_read_b64 %0, %3\n\tds_read_b64 %1, %3 offset:8\n\tds_read_b32 %2, %3 offset:16\n\t"
                     "s_waitcnt lgkmcnt(0)"
                     : "=v"(a), "=v"(b), "=v"(c) : "v"(la));
        q0 = a.x, q1 = a.y, q2 = b.x, q3 = b.y, q4 = c;
      } else if (MODE == 3) {
        u32x2 a, b;
        u32 c;
        asm volatile("ds_read2_b32 %0, %3 offset1:1\n\tds_read2_b32 %1, %3 offset0:2 offset1:3\n\t"
                     "ds_read_b32 %2, %3 offset:16\n\ts_waitcnt lgkmcnt(0)"
                     : "=v"(a), "=v"(b), "=v"(c) : "v"(la));
        q0 = a.x, q1 = a.y, q2 = b.x, q3 = b.y, q4 = c;
      } else {
        u32x3 a;
        u32x2 b;
        asm volatile("ds_read_b96 %0, %2\n\tds_read_b64 %1, %2 offset:12\n\ts_waitcnt lgkmcnt(0)"
                     : "=v"(a), "=v"(b) : "v"(la));
        q0 = a.x, q1 = a.y, q2 = a.z, q3 = b.x, q4 = b.y;
      }
      const u32 s = (u32)o & 3u;
      v = u32x4{__builtin_amdgcn_alignbyte(q1, q0, s), __builtin_amdgcn_alignbyte(q2, q1, s),
                __builtin_amdgcn_alignbyte(q3, q2, s), __builtin_amdgcn_alignbyte(q4, q3, s)};
    }
    const u32 c = v.x ^ (v.y * 3u) ^ (v.z * 5u) ^ (v.w * 7u);
    if (it == 0) first = c;
    x = x * 1664525u + 1013904223u;   // independent gathers: a throughput test
    acc += c;
  }
  out[2 * (blockIdx.x * 1024 + threadIdx.x)] = acc;
  out[2 * (blockIdx.x * 1024 + threadIdx.x) + 1] = first;
}

template <int M>
float run(u32* d) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  k<M><<<256, 1024>>>(d, 1);
  hipDeviceSynchronize();
  float best = 1e9f;
  for (int r = 0; r < 3; r++) {
    hipEventRecord(a);
    k<M><<<256, 1024>>>(d, 1);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    best = ms < best ? ms : best;
  }
  return best;
}

int main() {
  const size_t per = 256 * 1024 * 2;
  u32* d;
  hipMalloc(&d, per * 4 * 5);
  const char* names[] = {"ship b64x3+sel+align", "b128 a4 + b32 + align", "b64x2 a4 + b32 + align",
                         "read2_b32 x2 + b32 + align", "b96 a4 + b64 a4 + align"};
  float ms[5] = {run<0>(d), run<1>(d + per), run<2>(d + 2 * per), run<3>(d + 3 * per), run<4>(d + 4 * per)};
  u32* o = new u32[per * 5];
  hipMemcpy(o, d, per * 4 * 5, hipMemcpyDeviceToHost);
  for (int m = 0; m < 5; m++) {
    size_t bad = 0;
    for (size_t t = 0; t < per; t++) bad += o[m * per + t] != o[t];
    printf("{\"variant\": \"%s\", \"ms\": %.4f, \"ns_per_wave_gather_per_cu\": %.3f, \"mismatch\": %zu}\n",
           names[m], ms[m], ms[m] * 1e6 / (16.0 * ITERS), bad);
  }
  return 0;
}
