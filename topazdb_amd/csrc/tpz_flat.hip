// tpz_flat.hip — the flat column layout (include/tpz_gpu.h, tpz_flat_layout): for every block
// of a batch, the entries, key bytes and value bytes its decode will write, and the exclusive
// prefix sums of the three, so that tpz_decode_blocks_flat can put every key of the batch into
// one dense key column and every value into one dense value column (BlockIterator's key() /
// value() of every entry, src/block/iterator.rs:63-83, back to back in iterator order).
//
// A block's reservation follows the reference's reads exactly:
//   tag dispatch and the CRC split (src/block/compress.rs:95-113, src/block.rs:49-51): a block
//   that is empty, carries another tag, or is shorter than its CRC reserves nothing;
//   Block::decode's n and offsets (src/block.rs:54-59): a payload too short for them reserves
//   nothing (MALFORMED);
//   every entry i (src/block/iterator.rs:74-82): its key bytes when the key reads whole, its
//   value bytes when the value does too (an unreadable key or value is empty, as in the
//   TPZ_BLOCK_BAD_ENTRY record, tpz_spill.hip parse).
// The CRC is not checked here: a block that fails it keeps its reservation, unwritten.
//
// One wave per block (4-wave workgroups, a grid covering the batch): the block is staged into
// the wave's LDS window with coalesced 16-byte loads, and lanes parse 64 entries at a time from
// LDS. Reading every block whole moves the batch once: the entry headers are spread over every
// 64-byte sector of a 4 KiB block anyway. (A persistent version, 16 waves per workgroup looping
// over blocks with the next block's loads in flight, took 0.87-0.88 ms per 2^20 4 KiB blocks
// against 0.73-0.74: profiles/r4/flat_layout.txt.)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tpz_internal.h"

namespace tpz {
namespace {

typedef uint32_t u32;
typedef uint64_t u64;

constexpr int kFlWin = 4352;                 // a0 (<= 15) + len <= kFlWin: staged
constexpr u32 kFlMaxLen = kFlWin - 16;
constexpr int kFlRounds = kFlWin / 1024 + 1;  // 5 x 1 KiB loads per wave

__device__ __forceinline__ u32 lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

__device__ __forceinline__ u32 wave_sum(u32 x) {
  for (u32 o = 1; o < 64; o <<= 1) x += __shfl_xor(x, o, 64);
  return x;
}

// Big-endian u16 at byte a of a byte array (bytes::Buf::get_u16).
__device__ __forceinline__ u32 be16(const uint8_t* p, u64 a) { return ((u32)p[a] << 8) | p[a + 1]; }

// The reservation of one block whose bytes are p[0 .. len): {n, K, V} (see the file comment).
struct Sizes {
  u32 n, k, v;
};
__device__ __forceinline__ Sizes block_sizes(const uint8_t* p, u64 len) {
  Sizes z{0, 0, 0};
  if (len < 5 || p[len - 1] != 1) return z;                 // compress.rs:96-113, block.rs:49
  const u64 P = len - 5;
  if (P < 2) return z;                                      // block.rs:54
  const u32 n = be16(p, 0);
  if (P < 2 + 2 * (u64)n) return z;                         // block.rs:56-59
  const u64 db = 2 + 2 * (u64)n, dl = P - db;
  const u32 lane = lane_id();
  u32 kt = 0, vt = 0;
  for (u32 g0 = 0; g0 < n; g0 += 64) {
    const u32 i = g0 + lane;
    if (i < n) {
      const u64 off = be16(p, 2 + 2 * (u64)i);                                 // iterator.rs:74
      if (off + 2 <= dl) {
        const u32 kl = be16(p, db + off);                                      // :77
        if (off + 2 + kl <= dl) {
          kt += kl;                                                            // :78
          if (off + 4 + kl <= dl) {
            const u32 vl = be16(p, db + off + 2 + kl);                         // :80
            if (off + 4 + kl + vl <= dl) vt += vl;                             // :81-82
          }
        }
      }
    }
  }
  z.n = n;
  z.k = wave_sum(kt);
  z.v = wave_sum(vt);
  return z;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t src_rsrc(const uint8_t* src, u64 lim, u64 start) {
  u64 rem = lim > start ? lim - start : 0;
  if (rem > 0x7FFFFFF0ull) rem = 0x7FFFFFF0ull;
  return __builtin_amdgcn_make_buffer_rsrc((void*)(src + start), (short)0, (int)rem, 0x00020000);
}

// One block per wave and no loop: 4-wave workgroups that exit after their blocks, a grid
// covering the batch (a looping wave waits for its own stores' acknowledgements at every next
// load, tools/ubench_bw.hip; the LDS per workgroup is 17 KiB, so up to 9 workgroups share a CU).
constexpr int kFlWaves = 4;
__global__ __launch_bounds__(256) void flat_sizes_kernel(const uint8_t* src, const u64* ext,
                                                          u64 src_bytes, u32 nb, u64* first) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kFlWaves * kFlWin];
  const u32 lane = lane_id(), wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* win = lds + wid * kFlWin;
  const u64 st = (u64)nb + 1;
  const u32 b = blockIdx.x * kFlWaves + wid;
  if (b >= nb) return;
  const u64 s = ext[b], e = ext[b + 1];
  Sizes z{0, 0, 0};
  if (e >= s) {
    if (e - s <= kFlMaxLen && e + 16 <= src_bytes) {
      const u64 ws = s & ~15ull, e16 = (e + 15) & ~15ull;
      const __amdgpu_buffer_rsrc_t rs = src_rsrc(src, e16, ws);
      uint4 v[kFlRounds];
#pragma unroll
      for (int r = 0; r < kFlRounds; r++)
        v[r] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (u32)(r * 1024 + lane * 16), 0, 0));
#pragma unroll
      for (int r = 0; r < kFlRounds; r++)
        if (r * 1024 + lane * 16 < (u32)kFlWin) *reinterpret_cast<uint4*>(win + r * 1024 + lane * 16) = v[r];
      __builtin_amdgcn_wave_barrier();
      z = block_sizes(win + (s & 15u), e - s);
    } else {
      z = block_sizes(src + s, e - s);   // long blocks, and a block at the buffer's end
    }
  }
  if (lane == 0) {
    first[b] = z.n;
    first[st + b] = z.k;
    first[2 * st + b] = z.v;
  }
}

constexpr u32 kScPer = 4;                 // elements per thread
constexpr u32 kScWg = 256 * kScPer;       // elements per workgroup

__device__ __forceinline__ u64 wg_inclusive(u64 v, u64* wsum) {
  const u32 lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (u32 o = 1; o < 64; o <<= 1) {
    const u64 t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  if (lane == 63) wsum[w] = v;
  __syncthreads();
  for (u32 i = 0; i < w; i++) v += wsum[i];
  return v;
}

// Workgroup totals of array y (blockIdx.y) into part[y * (np + 1) + blockIdx.x].
__global__ __launch_bounds__(256) void flat_scan_parts(const u64* first, u32 nb, u64* part, u32 np) {
  __shared__ u64 wsum[4];
  const u64* a = first + (u64)blockIdx.y * (nb + 1);
  const u64 i0 = (u64)blockIdx.x * kScWg + threadIdx.x * kScPer;
  u64 s = 0;
  for (u32 j = 0; j < kScPer; j++)
    if (i0 + j < nb) s += a[i0 + j];
  s = wg_inclusive(s, wsum);
  if (threadIdx.x == 255) part[(u64)blockIdx.y * (np + 1) + blockIdx.x] = s;
}

// Exclusive scan of each array's workgroup totals in place, its total at part[.. + np].
__global__ __launch_bounds__(1024) void flat_scan_totals(u64* part, u32 np) {
  __shared__ u64 acc[1024];
  u64* pa = part + (u64)blockIdx.x * (np + 1);
  const u32 t = threadIdx.x, per = (np + 1023) / 1024;
  const u32 lo = min(np, t * per), hi = min(np, lo + per);
  u64 s = 0;
  for (u32 i = lo; i < hi; i++) s += pa[i];
  acc[t] = s;
  __syncthreads();
  for (u32 o = 1; o < 1024; o <<= 1) {
    const u64 v = t >= o ? acc[t - o] : 0;
    __syncthreads();
    acc[t] += v;
    __syncthreads();
  }
  u64 run = t ? acc[t - 1] : 0;
  for (u32 i = lo; i < hi; i++) {
    const u64 x = pa[i];
    pa[i] = run;
    run += x;
  }
  if (t == 1023) pa[np] = acc[1023];
}

// In place: a[i] = sum of a[j < i], a[nb] = the total.
__global__ __launch_bounds__(256) void flat_scan_write(u64* first, u32 nb, const u64* part, u32 np) {
  __shared__ u64 wsum[4];
  u64* a = first + (u64)blockIdx.y * (nb + 1);
  const u64* pa = part + (u64)blockIdx.y * (np + 1);
  const u64 i0 = (u64)blockIdx.x * kScWg + threadIdx.x * kScPer;
  u64 c[kScPer];
  u64 s = 0;
  for (u32 j = 0; j < kScPer; j++) {
    c[j] = i0 + j < nb ? a[i0 + j] : 0;
    s += c[j];
  }
  u64 run = wg_inclusive(s, wsum) - s + pa[blockIdx.x];
  for (u32 j = 0; j < kScPer; j++) {
    if (i0 + j < nb) a[i0 + j] = run;
    run += c[j];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) a[nb] = pa[np];
}

}  // namespace

uint64_t flat_scan_parts_words(uint32_t n_blocks) {
  return 3 * ((uint64_t)(n_blocks + kScWg - 1) / kScWg + 1);
}

void launch_scan_u64(u64* a, u32 n, u64* part, hipStream_t stream) {
  if (n == 0) {
    (void)hipMemsetAsync(a, 0, 8, stream);
    return;
  }
  const u32 np = (n + kScWg - 1) / kScWg;
  hipLaunchKernelGGL(flat_scan_parts, dim3(np, 1), dim3(256), 0, stream, a, n, part, np);
  hipLaunchKernelGGL(flat_scan_totals, dim3(1), dim3(1024), 0, stream, part, np);
  hipLaunchKernelGGL(flat_scan_write, dim3(np, 1), dim3(256), 0, stream, a, n, part, np);
}

void launch_flat_layout(const uint8_t* src, const u64* ext, u64 src_bytes, u32 n_blocks,
                        u64* first, u64* part, u32 num_cus, hipStream_t stream) {
  if (n_blocks == 0) {
    (void)hipMemsetAsync(first, 0, 3 * 8, stream);
    return;
  }
  hipLaunchKernelGGL(flat_sizes_kernel, dim3((n_blocks + kFlWaves - 1) / kFlWaves), dim3(256), 0,
                     stream, src, ext, src_bytes, n_blocks, first);
  const u32 np = (n_blocks + kScWg - 1) / kScWg;
  hipLaunchKernelGGL(flat_scan_parts, dim3(np, 3), dim3(256), 0, stream, first, n_blocks, part, np);
  hipLaunchKernelGGL(flat_scan_totals, dim3(3), dim3(1024), 0, stream, part, np);
  hipLaunchKernelGGL(flat_scan_write, dim3(np, 3), dim3(256), 0, stream, first, n_blocks, part, np);
}

}  // namespace tpz
