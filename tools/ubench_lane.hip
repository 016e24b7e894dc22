// Diagnostic (not shipped): cost of per-lane scattered 16-byte accesses, the memory pattern of a
// one-block-per-lane codec. Each lane streams through its own 4 KiB region (2^18 lanes, 1 GiB):
//   ld_al / ld_mis   16-byte loads at 16-byte aligned / misaligned (+3) addresses
//   st_al / st_mis   16-byte stores, aligned / misaligned
//   cp_al / cp_mis   load + store (a lane-wise copy), aligned / misaligned
//   ld4_al           4-byte loads (aligned)
//   ld_oob75         buffer loads, 3 of 4 lanes at an out-of-range offset (a masked-off piece)
//   ld_exec25        the same loads with 3 of 4 lanes switched off by the exec mask
//   ld_buf           buffer loads, every lane in range
//   st_line8/4       each group of 8 (4) lanes stores one whole 128-byte (64-byte) line of its
//                    group's region per instruction (a wave flushing 8 (16) blocks' lines)
// Prints one JSON line per variant: median ms and lane accesses per ns.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

typedef unsigned __int128 u128;
#define CHECK(x)                                                          \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      return 1;                                                           \
    }                                                                     \
  } while (0)

constexpr uint32_t kRegion = 4096, kLanes = 1u << 18, kSteps = 250;   // 250 x 16 B < 4096 - 16

template <int MODE, int MIS>
__global__ __launch_bounds__(256) void k(uint8_t* a, uint8_t* b, uint32_t* sink) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  uint8_t* pa = a + (uint64_t)t * kRegion + MIS;
  uint8_t* pb = b + (uint64_t)t * kRegion + MIS;
  uint32_t acc = 0;
  for (uint32_t i = 0; i < kSteps; i++) {
    if (MODE == 0) {
      u128 v;
      __builtin_memcpy(&v, pa + 16 * i, 16);
      acc ^= (uint32_t)v;
    } else if (MODE == 1) {
      const u128 v = ((u128)i << 64) | t;
      __builtin_memcpy(pb + 16 * i, &v, 16);
    } else if (MODE == 2) {
      u128 v;
      __builtin_memcpy(&v, pa + 16 * i, 16);
      __builtin_memcpy(pb + 16 * i, &v, 16);
    } else if (MODE == 6 || MODE == 7 || MODE == 8) {
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a, (short)0, 0x7FFFFFF0, 0x00020000);
      const uint32_t off = (uint32_t)((uint64_t)t * kRegion + 16 * i) & 0x3FFFFFFFu;
      const bool on = MODE == 8 || (t & 3) == 0;
      if (MODE == 7) {
        if (on) acc ^= (uint32_t)__builtin_bit_cast(u128, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
      } else {
        acc ^= (uint32_t)__builtin_bit_cast(u128, __builtin_amdgcn_raw_buffer_load_b128(rs, on ? off : 0x80000000u, 0, 0));
      }
    } else if (MODE == 4 || MODE == 5) {
      // G lanes per line: region of the group, line i of it; lane's 16-byte piece
      constexpr uint32_t G = MODE == 4 ? 8 : 4;
      const uint32_t grp = t / G, sub = t % G;
      uint8_t* base = b + (uint64_t)grp * kRegion * G;
      const u128 v = ((u128)i << 64) | t;
      // G x 4 KiB per group: 250 x 16 G bytes = 250 lines of 16 G bytes
      __builtin_memcpy(base + (uint64_t)i * 16 * G + 16 * sub, &v, 16);
    } else {
      uint32_t v;
      __builtin_memcpy(&v, pa + 16 * i, 4);
      acc ^= v;
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char** argv) {
  std::vector<std::string> vars;
  for (int i = 1; i < argc; i++) vars.push_back(argv[i]);
  if (vars.empty()) vars = {"ld_al", "ld_mis", "st_al", "st_mis", "cp_al", "cp_mis", "ld4_al", "st_line8", "st_line4", "st_al"};
  const uint64_t N = (uint64_t)kLanes * kRegion;
  uint8_t *a, *b;
  uint32_t* s;
  CHECK(hipMalloc(&a, N));
  CHECK(hipMalloc(&b, N));
  CHECK(hipMalloc(&s, 4));
  CHECK(hipMemset(a, 1, N));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (const std::string& v : vars) {
    auto launch = [&]() {
      dim3 g(kLanes / 256), bl(256);
      if (v == "ld_al") k<0, 0><<<g, bl>>>(a, b, s);
      else if (v == "ld_mis") k<0, 3><<<g, bl>>>(a, b, s);
      else if (v == "st_al") k<1, 0><<<g, bl>>>(a, b, s);
      else if (v == "st_mis") k<1, 3><<<g, bl>>>(a, b, s);
      else if (v == "cp_al") k<2, 0><<<g, bl>>>(a, b, s);
      else if (v == "cp_mis") k<2, 3><<<g, bl>>>(a, b, s);
      else if (v == "ld4_al") k<3, 0><<<g, bl>>>(a, b, s);
      else if (v == "st_line8") k<4, 0><<<g, bl>>>(a, b, s);
      else if (v == "ld_oob75") k<6, 0><<<g, bl>>>(a, b, s);
      else if (v == "ld_exec25") k<7, 0><<<g, bl>>>(a, b, s);
      else if (v == "ld_buf") k<8, 0><<<g, bl>>>(a, b, s);
      else if (v == "st_line4") k<5, 0><<<g, bl>>>(a, b, s);
    };
    for (int w = 0; w < 2; w++) launch();
    CHECK(hipDeviceSynchronize());
    std::vector<float> ms;
    for (int r = 0; r < 9; r++) {
      CHECK(hipEventRecord(e0));
      launch();
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float t;
      CHECK(hipEventElapsedTime(&t, e0, e1));
      ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    const double acc = (double)kLanes * kSteps * (v.rfind("cp", 0) == 0 ? 2 : 1);
    printf("{\"variant\": \"%s\", \"ms_median\": %.4f, \"lane_accesses_per_ns\": %.2f, \"gb_s\": %.1f}\n",
           v.c_str(), ms[4], acc / (ms[4] * 1e6), acc * (v == "ld4_al" ? 4 : 16) / (ms[4] * 1e6));
    fflush(stdout);
  }
  return 0;
}
