// Diagnostic (not shipped): VALU issue rate per SIMD on gfx950, to read SQ_ACTIVE_INST_VALU
// against a ceiling. W waves per CU (W/4 per SIMD) each run a loop of independent 32-bit
// integer ops (8 independent chains, v_bitop3 / v_add / v_lshlrev_sdwa-like byte shifts);
// prints VALU wave-instructions per SIMD per shader clock (s_memtime) and per ns.
//   ubench_valu            all shapes
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

typedef uint32_t u32;
typedef uint64_t u64;

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      return 1;                                                               \
    }                                                                         \
  } while (0)

constexpr int kIters = 4096;

// 8 chains per iteration: 40 VALU (KIND 0) / 64 VALU (KIND 1) per iteration in the ISA
template <int KIND>
__global__ void valu_k(u32* out, u64* clk, u32 seed) {
  u32 a[8];
#pragma unroll
  for (int i = 0; i < 8; i++) a[i] = threadIdx.x * 7 + i + seed;
  const u64 t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIters; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      if (KIND == 0) {
        a[i] = __builtin_amdgcn_bitop3_b32(a[i], a[(i + 1) & 7], 0x9E3779B9u, 0x96);
        a[i] = a[i] + 0x7F4A7C15u;
        a[i] = __builtin_amdgcn_bitop3_b32(a[i], a[(i + 3) & 7], 0x85EBCA6Bu, 0x96);
        a[i] = a[i] ^ (a[i] >> 13);
      } else {
        // byte extract shifted by 2 (the CRC lookup's address op) + xor3
        a[i] = ((a[i] >> 8) & 0xFFu) << 2 | (a[i] & 0xFFFFFC00u);
        a[i] = __builtin_amdgcn_bitop3_b32(a[i], a[(i + 1) & 7], 0x9E3779B9u, 0x96);
        a[i] = ((a[i] >> 16) & 0xFFu) << 2 | (a[i] & 0xFFFFFC00u);
        a[i] = __builtin_amdgcn_bitop3_b32(a[i], a[(i + 5) & 7], 0x85EBCA6Bu, 0x96);
      }
    }
  }
  const u64 t1 = __builtin_amdgcn_s_memtime();
  u32 r = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r ^= a[i];
  if (r == 0x12345678u) out[0] = r;
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  u32* out;
  u64* clk;
  CHECK(hipMalloc(&out, 4));
  CHECK(hipMalloc(&clk, 8 * 65536));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int shapes[] = {4, 8, 16, 32};
  for (int kind = 0; kind < 2; kind++) {
    for (int w : shapes) {
      // w waves per CU: one workgroup of 64*w threads per CU (w <= 16), two for 32
      const int wg = w <= 16 ? 64 * w : 1024;
      const int grid = w <= 16 ? cus : 2 * cus;
      auto launch = [&]() {
        if (kind == 0) valu_k<0><<<grid, wg>>>(out, clk, 1);
        else valu_k<1><<<grid, wg>>>(out, clk, 1);
      };
      launch();
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(e0));
      const int reps = 5;
      for (int r = 0; r < reps; r++) launch();
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      ms /= reps;
      u64 h[2];
      CHECK(hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost));
      // VALU wave-instructions per SIMD: w/4 waves x kIters x 32
      const double per_simd = (double)w / 4 * kIters * (kind == 0 ? 40 : 64);  // VALU per iteration, from the ISA
      printf("{\"kind\": %d, \"waves_per_cu\": %d, \"ms\": %.4f, \"clk_wg0\": %llu, "
             "\"valu_per_simd_per_clk\": %.3f, \"valu_per_simd_per_ns\": %.3f}\n",
             kind, w, ms, (unsigned long long)h[0], per_simd / (double)h[0], per_simd / (ms * 1e6));
    }
  }
  return 0;
}
