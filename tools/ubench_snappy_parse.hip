// ubench_snappy_parse.hip — diagnostic: the element-boundary discovery of a
// block-parallel snappy decode, alone, timed against the ring kernel's whole codec step.
//
// A snappy block (compress.rs:104-107) is a varint preamble and a chain of elements; element i+1
// starts where element i ends, so the ring kernel (tpz_codec.hip) walks the chain one element per
// trip, one block per lane. A decode with a wave per block needs the chain's positions first. This
// probe finds them with 64 lanes:
//   1. the block's stream is staged in LDS; every position p gets next(p) = p + the size of the
//      element a header at p would describe (speculative: most positions are not element starts);
//   2. the stream is cut into 64 segments, one per lane; lane l computes, for every position p of
//      its segment, the first chain position at or past the segment's end when the chain enters
//      the segment at p: E(p) = next(p) if that is past the end, else E(next(p)) (downwards, so
//      E(next(p)) is already known);
//   3. the wave follows the chain from the preamble's end through E, one segment at a time: the
//      entry position of every segment (64 dependent LDS reads);
//   4. each lane walks its segment from its entry and counts the element starts.
// Output: the element count per block (0 for a stream whose chain does not end at the stream's
// end), checked against one thread per block walking the chain (ref kernel).
//
// Build: hipcc -O3 --offload-arch=gfx950 -shared -fPIC -o tools/libubench_snappy_parse.so
//        tools/ubench_snappy_parse.hip   (tools/snappy_parse_probe.py builds and runs it)
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32;
typedef uint64_t u64;

constexpr int kWaves = 10;         // waves per workgroup (one workgroup per CU: the LDS)
constexpr int kMaxN = 3072;        // stream bytes a wave stages (4kc blocks compress to ~2.8 KB)
constexpr int kSlot = kMaxN + 16 + 2 * (kMaxN + 8) * 2;   // bytes | next (u16) | exit (u16)

__device__ __forceinline__ u32 lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// The size of the element whose tag byte is at s[i] (bytes past n read as 0): snappy's literal
// (1-4 length bytes after tags 60-63) and copy-1/2/4 elements.
__device__ __forceinline__ u32 elem_size(const uint8_t* s, u32 i) {
  const u32 tag = s[i], kind = tag & 3, t6 = tag >> 2;
  if (kind == 1) return 2;
  if (kind == 2) return 3;
  if (kind == 3) return 5;
  if (t6 < 60) return 1 + t6 + 1;
  const u32 nb = t6 - 59;
  u32 l = s[i + 1];
  if (nb > 1) l |= (u32)s[i + 2] << 8;
  if (nb > 2) l |= (u32)s[i + 3] << 16;
  if (nb > 3) l |= (u32)s[i + 4] << 24;
  const u64 sz = 1ull + nb + (u64)l + 1;
  return sz > 0xFFFFu ? 0xFFFFu : (u32)sz;
}

__device__ __forceinline__ u32 preamble(const uint8_t* s, u32 n) {
  for (u32 i = 0; i < 10 && i < n; i++)
    if (!(s[i] & 0x80)) return i + 1;
  return 0;
}

__global__ __launch_bounds__(64 * kWaves) void parse_kernel(const uint8_t* src, const u64* ext,
                                                            u32 nb, u32* count) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kWaves * kSlot];
  const u32 lane = lane_id(), wid = threadIdx.x >> 6;
  uint8_t* W = lds + wid * kSlot;
  uint16_t* NX = reinterpret_cast<uint16_t*>(W + kMaxN + 16);
  uint16_t* EX = NX + kMaxN + 8;
  for (u32 b = blockIdx.x * kWaves + wid; b < nb; b += gridDim.x * kWaves) {
    const u64 s0 = ext[b], e0 = ext[b + 1];
    const u32 n = (u32)(e0 - s0) - 1;            // the stream without the tag byte
    if (e0 - s0 < 2 || n > kMaxN) {
      if (lane == 0) count[b] = 0;
      continue;
    }
    // 1. stage (byte loads, coalesced per 64 bytes), pad with zeros
    for (u32 i = lane; i < n + 16; i += 64) W[i] = i < n ? src[s0 + i] : 0;
    __builtin_amdgcn_wave_barrier();
    const u32 h = __builtin_amdgcn_readfirstlane(preamble(W, n));
    const u32 L = n;                            // positions h .. L-1; L is the end
    for (u32 p = h + lane; p < L; p += 64) {
      const u32 nx = p + elem_size(W, p);
      NX[p] = (uint16_t)(nx > L ? L + 1 : nx);  // L + 1: past the end (invalid)
    }
    __builtin_amdgcn_wave_barrier();
    // 2. segment exits, downwards
    const u32 S = (L - h + 63) / 64;
    const u32 lo = h + lane * S, hi = min(L, lo + S);
    for (u32 p = hi; p-- > lo;) {
      const u32 nx = NX[p];
      EX[p] = (uint16_t)(nx >= hi ? nx : EX[nx]);
    }
    __builtin_amdgcn_wave_barrier();
    // 3. the chain through the segments: entry of each segment (wave-uniform walk)
    u32 x = h, my_entry = 0xFFFFu;
    u32 seg = 0;
    bool ok = h != 0;
    while (ok && x < L) {
      seg = (x - h) / S;
      if (lane == seg) my_entry = x;
      x = EX[x];
      x = __builtin_amdgcn_readfirstlane(x);
    }
    ok = ok && x == L;
    // 4. count the element starts in each segment
    u32 c = 0;
    if (ok && my_entry != 0xFFFFu) {
      for (u32 p = my_entry; p < hi; p = NX[p]) c++;
    }
    for (u32 o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o);
    if (lane == 0) count[b] = ok ? c : 0u;
    __builtin_amdgcn_wave_barrier();
  }
}

// Reference: one thread per block walks the chain from global memory.
__global__ __launch_bounds__(256) void ref_kernel(const uint8_t* src, const u64* ext, u32 nb,
                                                  u32* count) {
  const u32 b = blockIdx.x * 256 + threadIdx.x;
  if (b >= nb) return;
  const u64 s0 = ext[b], e0 = ext[b + 1];
  if (e0 - s0 < 2) { count[b] = 0; return; }
  const uint8_t* s = src + s0;
  const u32 n = (u32)(e0 - s0) - 1;
  u64 p = preamble(s, n);
  u32 c = 0;
  const bool ok0 = p != 0;
  while (ok0 && p < n) {
    const u32 tag = s[p], kind = tag & 3, t6 = tag >> 2;
    u64 sz;
    if (kind == 1) sz = 2;
    else if (kind == 2) sz = 3;
    else if (kind == 3) sz = 5;
    else if (t6 < 60) sz = t6 + 2;
    else {
      const u32 nb2 = t6 - 59;
      u64 l = 0;
      for (u32 k = 0; k < nb2; k++) l |= (u64)(p + 1 + k < n ? s[p + 1 + k] : 0) << (8 * k);
      sz = 1 + nb2 + l + 1;
    }
    p += sz;
    c++;
  }
  count[b] = (ok0 && p == n) ? c : 0u;
}

extern "C" int probe_parse(const uint8_t* src, const u64* ext, u32 nb, u32* count, int num_cus,
                           void* stream) {
  const u32 grid = (u32)num_cus;
  hipLaunchKernelGGL(parse_kernel, dim3(grid), dim3(64 * kWaves), 0, (hipStream_t)stream,
                     src, ext, nb, count);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
extern "C" int probe_ref(const uint8_t* src, const u64* ext, u32 nb, u32* count, void* stream) {
  hipLaunchKernelGGL(ref_kernel, dim3((nb + 255) / 256), dim3(256), 0, (hipStream_t)stream, src, ext,
                     nb, count);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
