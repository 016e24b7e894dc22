// Diagnostic (not shipped): the memory skeleton of the 4k decode, without the decode.
// 2^20 blocks of 4155 B back to back (unaligned starts); per block the decoder reads the block
// (5 x 1 KiB wave loads, the last partial) and writes 31 whole 128-B lines of stream at the slot
// base plus 3 lines of entry ends. Variants differ only in how loads and stores are scheduled:
//   copy        grid-stride 16-B copy of the same byte count (4 loads in flight per lane)
//   d1          one wave per block, next block's loads issued before this block's stores; the
//               number of stores is made data-dependent (as in the decoder), so the wait for
//               the prefetch is vmcnt(0) and also drains this block's stores
//   d1c         the same with a fixed store count: the compiler's wait is vmcnt(#stores)
//   d2c         two blocks of loads in flight per wave (fixed store count)
//   lds         loads by LDS-DMA (global_load_lds_dwordx4) into a per-wave double buffer
// Usage: ubench_skel [variant ...]; prints one JSON line per variant.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <cstring>
#include <algorithm>
#include <string>
#include <vector>

typedef uint32_t u32;
typedef uint64_t u64;
constexpr u32 NB = 1u << 20, BL = 4155, NLINES = 31, ELINES = 3;

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                     \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

__device__ __forceinline__ u64 slot_base(u64 e, u64 i) { return ((e + 127) & ~127ull) + 256 * i; }
__device__ __forceinline__ u64 ends_base(u64 e, u64 i) { return 16 * (e / 96 + i) * 8; }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, u32 n) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)n, 0x00020000);
}
typedef u32 u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void copy_kernel(const uint4* __restrict__ s, uint4* __restrict__ d,
                                                   u64 n16) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const uint4 a = s[i], b = s[i + stride], c = s[i + 2 * stride], e = s[i + 3 * stride];
    d[i] = a;
    d[i + stride] = b;
    d[i + 2 * stride] = c;
    d[i + 3 * stride] = e;
  }
  for (; i < n16; i += stride) d[i] = s[i];
}

// one wave per block, prefetch depth D; VARIABLE: store count read from memory (opaque);
// WORK: VALU instructions per block (4 independent chains), LDSW: random ds_read_b32 per block
// META: 0 none; 1 per-block status byte + count + crc stores (the decoder's put_meta);
// CONTIG: each workgroup takes a contiguous range of blocks (else round-robin over workgroups)
template <int D, bool VARIABLE, int WAVES, int WORK = 0, int LDSW = 0, int META = 0, bool CONTIG = false>
__global__ __launch_bounds__(64 * WAVES) void skel_kernel(const uint8_t* src, uint8_t* out,
                                                          uint8_t* ends, const u32* nlines_p,
                                                          uint8_t* meta = nullptr) {
  __shared__ u32 tab[LDSW ? 16384 : 1];
  if (LDSW) {
    for (u32 i = threadIdx.x; i < 16384; i += blockDim.x) tab[i] = i * 2654435761u;
    __syncthreads();
  }
  const u32 lane = threadIdx.x & 63;
  const u32 wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 nw = gridDim.x * WAVES;
  const u32 nlines = VARIABLE ? __builtin_amdgcn_readfirstlane(*nlines_p) : NLINES;
  const u32 per = (NB + gridDim.x - 1) / gridDim.x;
  const u32 bend = CONTIG ? min(NB, (blockIdx.x + 1) * per) : NB;
  u32 b = CONTIG ? blockIdx.x * per + wid : blockIdx.x * WAVES + wid;
  const u32 nw_eff = CONTIG ? WAVES : nw;
  uint4 v[D][5];
  auto issue = [&](u32 bb, uint4* dst) {
    if (bb >= bend) return;
    const u64 s = (u64)bb * BL, ws = s & ~15ull, e = s + BL;
    const __amdgpu_buffer_rsrc_t r = rsrc(src + ws, (u32)(((e + 15) & ~15ull) - ws));
#pragma unroll
    for (int q = 0; q < 5; q++)
      dst[q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, q * 1024 + lane * 16, 0, 0));
  };
#pragma unroll
  for (int d = 0; d < D; d++) issue(b + d * nw_eff, v[d]);
  u32 acc = 0;
  while (b < bend) {
    uint4 cur[5];
#pragma unroll
    for (int q = 0; q < 5; q++) cur[q] = v[0][q];
#pragma unroll
    for (int d = 0; d + 1 < D; d++)
#pragma unroll
      for (int q = 0; q < 5; q++) v[d][q] = v[d + 1][q];
    issue(b + D * nw_eff, v[D - 1]);
    // "decode": fold the block into the stores
    const u64 s = (u64)b * BL;
    const __amdgpu_buffer_rsrc_t ro = rsrc(out + slot_base(s, b), NLINES * 128);
    for (u32 l = 0; l < (nlines * 8 + 63) / 64; l++) {      // 31 lines = 248 chunks = 4 stores
      uint4 x = cur[l];
      x.x ^= acc;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, x), ro, l * 1024 + lane * 16, 0, 0);
    }
    const __amdgpu_buffer_rsrc_t re = rsrc(ends + ends_base(s, b), ELINES * 128);
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) u32,
                                                             make_uint2(cur[4].x, lane)),
                                          re, lane * 8, 0, 0);
    acc += cur[4].y;
    if (META) {
      const bool l0 = lane == 0;
      const __amdgpu_buffer_rsrc_t rm = rsrc(meta, 0x7FFFFFF0);
      __builtin_amdgcn_raw_buffer_store_b8((uint8_t)acc, rm, l0 ? b : 0x7FFFFFF8u, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32(acc, rm, l0 ? NB + 4 * b : 0x7FFFFFF8u, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32(acc + 1, rm, l0 ? 5 * NB + 4 * b : 0x7FFFFFF8u, 0, 0);
    }
    if (WORK) {
      u32 x0 = cur[0].x, x1 = cur[1].y, x2 = cur[2].z, x3 = cur[3].w;
#pragma unroll 8
      for (int w = 0; w < WORK / 8; w++) {
        x0 = x0 * 0x9E3779B1u + 7u;
        x1 = x1 * 0x85EBCA77u + 3u;
        x2 = x2 * 0xC2B2AE3Du + 5u;
        x3 = x3 * 0x27D4EB2Fu + 1u;
      }
      acc ^= x0 ^ x1 ^ x2 ^ x3;
    }
    if (LDSW) {
      u32 y = cur[1].x ^ lane * 77u;
#pragma unroll 4
      for (int w = 0; w < LDSW; w++) y = tab[(y ^ (y >> 9)) & 16383] + w;
      acc ^= y;
    }
    b += nw_eff;
  }
  if (acc == 0x12345678u) out[0] = 1;
}

// LDS-DMA variant: per wave two 4.4 KiB buffers; the loads of block k+1 land in LDS while block
// k's stores (read back from LDS) go out. WAVES waves per workgroup, one workgroup per CU.
template <int WAVES>
__global__ __launch_bounds__(64 * WAVES) void lds_kernel(const uint8_t* src, uint8_t* out, uint8_t* ends) {
  constexpr u32 kBuf = 5 * 1024;
  __shared__ __attribute__((aligned(16))) uint8_t lds[WAVES * 2 * kBuf];
  const u32 lane = threadIdx.x & 63;
  const u32 wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 nw = gridDim.x * WAVES;
  uint8_t* buf0 = lds + wid * 2 * kBuf;
  u32 b = blockIdx.x * WAVES + wid;
  auto issue = [&](u32 bb, uint8_t* dst) {
    if (bb >= NB) return;
    const u64 s = (u64)bb * BL, ws = s & ~15ull;
#pragma unroll
    for (int q = 0; q < 5; q++)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + ws + q * 1024 + lane * 16),
                                       (__attribute__((address_space(3))) void*)(dst + q * 1024),
                                       16, 0, 0);
  };
  u32 k = 0;
  issue(b, buf0);
  u32 acc = 0;
  while (b < NB) {
    uint8_t* cur = buf0 + (k & 1) * kBuf;
    uint8_t* nxt = buf0 + ((k + 1) & 1) * kBuf;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");        // block k landed (and k-1's stores)
    issue(b + nw, nxt);
    const u64 s = (u64)b * BL;
    const __amdgpu_buffer_rsrc_t ro = rsrc(out + slot_base(s, b), NLINES * 128);
#pragma unroll
    for (u32 l = 0; l < 4; l++) {
      uint4 x = *reinterpret_cast<const uint4*>(cur + l * 1024 + lane * 16);
      x.x ^= acc;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, x), ro, l * 1024 + lane * 16, 0, 0);
    }
    const uint4 t = *reinterpret_cast<const uint4*>(cur + 4 * 1024 + lane * 16);
    const __amdgpu_buffer_rsrc_t re = rsrc(ends + ends_base(s, b), ELINES * 128);
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) u32,
                                                             make_uint2(t.x, lane)),
                                          re, lane * 8, 0, 0);
    acc += t.y;
    b += nw;
    k++;
  }
  if (acc == 0x12345678u) out[0] = 1;
}

int main(int argc, char** argv) {
  std::vector<std::string> vars;
  for (int i = 1; i < argc; i++) vars.push_back(argv[i]);
  if (vars.empty()) vars = {"copy", "d1", "d1c", "d2c", "d1c_w8", "d2c_w8", "d1c_2wg", "lds16", "lds8"};
  const u64 in_bytes = (u64)NB * BL;
  const u64 out_cap = ((in_bytes + 127) & ~127ull) + 256ull * NB + 4096;
  const u64 ends_cap = 16ull * (in_bytes / 96 + NB) * 8 + 4096;
  uint8_t *src, *out, *ends;
  u32* nl;
  CHECK(hipMalloc(&src, in_bytes + 4096));
  CHECK(hipMalloc(&out, out_cap));
  CHECK(hipMalloc(&ends, ends_cap));
  CHECK(hipMalloc(&nl, 4));
  uint8_t* meta;
  CHECK(hipMalloc(&meta, 9ull * NB + 4096));
  CHECK(hipMemset(src, 0x5A, in_bytes + 4096));
  const u32 nlines = NLINES;
  CHECK(hipMemcpy(nl, &nlines, 4, hipMemcpyHostToDevice));
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const u32 cus = prop.multiProcessorCount;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const double moved = (double)NB * (BL + NLINES * 128 + ELINES * 128);   // bytes per launch
  for (const std::string& v : vars) {
    auto launch = [&]() {
      // copy: in_bytes read + in_bytes written (both buffers hold at least in_bytes)
      if (v == "copy") copy_kernel<<<cus * 8, 256>>>((const uint4*)src, (uint4*)out, in_bytes / 16);
      else if (v == "d1") skel_kernel<1, true, 16><<<cus, 1024>>>(src, out, ends, nl);
      else if (v == "d1c") skel_kernel<1, false, 16><<<cus, 1024>>>(src, out, ends, nl);
      else if (v == "d2c") skel_kernel<2, false, 16><<<cus, 1024>>>(src, out, ends, nl);
      else if (v == "d3c") skel_kernel<3, false, 16><<<cus, 1024>>>(src, out, ends, nl);
      else if (v == "d1c_w8") skel_kernel<1, false, 8><<<cus, 512>>>(src, out, ends, nl);
      else if (v == "d2c_w8") skel_kernel<2, false, 8><<<cus, 512>>>(src, out, ends, nl);
      else if (v == "d1c_2wg") skel_kernel<1, false, 16><<<cus * 2, 1024>>>(src, out, ends, nl);
      else if (v == "d2c_2wg") skel_kernel<2, false, 16><<<cus * 2, 1024>>>(src, out, ends, nl);
      else if (v == "w200") skel_kernel<1, false, 16, 200><<<cus, 1024>>>(src, out, ends, nl);
      else if (v == "w400") skel_kernel<1, false, 16, 400><<<cus, 1024>>>(src, out, ends, nl);
      else if (v == "w700") skel_kernel<1, false, 16, 700><<<cus, 1024>>>(src, out, ends, nl);
      else if (v == "w1000") skel_kernel<1, false, 16, 1000><<<cus, 1024>>>(src, out, ends, nl);
      else if (v == "w700d2") skel_kernel<2, false, 16, 700><<<cus, 1024>>>(src, out, ends, nl);
      else if (v == "w700v") skel_kernel<1, true, 16, 700><<<cus, 1024>>>(src, out, ends, nl);
      else if (v == "l40") skel_kernel<1, false, 16, 0, 40><<<cus, 1024>>>(src, out, ends, nl);
      else if (v == "l80") skel_kernel<1, false, 16, 0, 80><<<cus, 1024>>>(src, out, ends, nl);
      else if (v == "w400l40") skel_kernel<1, false, 16, 400, 40><<<cus, 1024>>>(src, out, ends, nl);
      else if (v == "w700l80") skel_kernel<1, false, 16, 700, 80><<<cus, 1024>>>(src, out, ends, nl);
      else if (v == "meta") skel_kernel<1, false, 16, 0, 0, 1, false><<<cus, 1024>>>(src, out, ends, nl, meta);
      else if (v == "meta_contig") skel_kernel<1, false, 16, 0, 0, 1, true><<<cus, 1024>>>(src, out, ends, nl, meta);
      else if (v == "contig") skel_kernel<1, false, 16, 0, 0, 0, true><<<cus, 1024>>>(src, out, ends, nl, meta);
      else if (v == "lds16") lds_kernel<16><<<cus, 1024>>>(src, out, ends);
      else if (v == "lds8") lds_kernel<8><<<cus, 512>>>(src, out, ends);
      else if (v == "lds12") lds_kernel<12><<<cus, 768>>>(src, out, ends);
    };
    for (int w = 0; w < 5; w++) launch();
    CHECK(hipDeviceSynchronize());
    const int reps = 20;
    std::vector<float> ms;
    for (int r = 0; r < reps; r++) {
      CHECK(hipEventRecord(e0));
      launch();
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float t;
      CHECK(hipEventElapsedTime(&t, e0, e1));
      ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    const float med = ms[reps / 2];
    const double bytes = v == "copy" ? 2.0 * in_bytes : moved;
    printf("{\"variant\": \"%s\", \"ms_median\": %.4f, \"ms_min\": %.4f, \"tb_s\": %.3f}\n", v.c_str(), med,
           ms[0], bytes / (med * 1e-3) / 1e12);
    fflush(stdout);
  }
  return 0;
}
