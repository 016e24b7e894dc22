// Microbenchmark: LDS lookup instruction throughput on gfx950 (diagnostic, not shipped).
// 256 workgroups x 1024 threads; each thread does ITERS x 16 independent lookups.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
constexpr int ITERS = 4096;
template <int MODE>
__global__ __launch_bounds__(1024, 4) void k(uint32_t* out, uint32_t seed) {
  __shared__ uint32_t tab[16 * 256 + 64];
  for (int i = threadIdx.x; i < 16 * 256; i += 1024) tab[i] = i * 2654435761u;
  __syncthreads();
  uint32_t lane = threadIdx.x & 63;
  uint32_t x = seed ^ (threadIdx.x * 0x9E3779B9u) ^ blockIdx.x;
  uint32_t acc = 0;
  uint32_t breg = x * 0x85ebca6bu;
  for (int it = 0; it < ITERS; it++) {
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) {
      uint32_t idx = (x >> ((j & 3) * 8)) & 0xFF;
      if (MODE == 0) c ^= tab[j * 256 + idx];                       // random byte-indexed
      if (MODE == 1) c ^= tab[j * 256 + ((lane + j) & 31) + 32 * (idx & 7)]; // lane->bank (conflict-free)
      if (MODE == 2) c ^= __builtin_amdgcn_ds_bpermute((int)((idx & 63) << 2), (int)(breg + j));
      if (MODE == 3) c ^= (uint32_t)__shfl(breg + j, idx & 63);
    }
    x = x * 1664525u + 1013904223u + c;
    acc ^= c;
  }
  out[blockIdx.x * 1024 + threadIdx.x] = acc;
}
template <int M> float run(uint32_t* d) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  k<M><<<256, 1024>>>(d, 1); hipDeviceSynchronize();
  hipEventRecord(a); k<M><<<256, 1024>>>(d, 2); hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b); return ms;
}
int main() {
  uint32_t* d; hipMalloc(&d, 256 * 1024 * 4);
  const char* names[] = {"ds_read_b32 random(256)", "ds_read_b32 lane->bank", "ds_bpermute random", "__shfl random"};
  float ms[4] = {run<0>(d), run<1>(d), run<2>(d), run<3>(d)};
  for (int m = 0; m < 4; m++) {
    double instr_per_cu = 16.0 * 16 * ITERS * 16;  // 16 waves/CU x ITERS x 16 lookups
    printf("%-28s %8.3f ms  %6.2f ns/wave-instr/CU  %5.2f cyc@2.35GHz\n", names[m], ms[m],
           ms[m] * 1e6 / instr_per_cu, ms[m] * 1e6 / instr_per_cu * 2.35);
  }
  return 0;
}
