// tpz_encode.hip — gfx950 kernels for the write side of the block path: SsTableBuilder's block
// cuts and Block::encode + checksum for a batch of sorted entries (compaction output,
// src/table/builder.rs:49-85; SURVEY.md §8f row 4's alternative).
//
//  plan    BlockBuilder::add (src/block/builder.rs:26-41): an entry joins the current block while
//          size + encode_len + 2 <= block_size (size = the block's entry bytes so far);
//          SsTableBuilder::add (src/table/builder.rs:49-64) starts the next block with the entry
//          that did not fit. The block starts are the chain 0 -> nx[0] -> ... over entries:
//            plan_next_kernel   nx[a] = entries of a block that starts at entry a (galloping
//                               search over the entries' prefix sums S staged in LDS, closed
//                               form from kpos/vpos)
//            plan_table_kernel  per chunk of C entries (C = max(2048, w)), the chain's exit offset into the
//                               next chunk for every entry offset it can enter at (< w, the
//                               longest block in entries)
//            plan_round_kernel  Hillis-Steele scan of those transfer tables (function
//                               composition, log2(chunks) rounds): the entry offset of every chunk
//            plan_count_kernel + plan_scan_kernel + plan_write_kernel: one walk per chunk counts
//                               and then writes its block starts and byte extents
//            (chunks of <= 8192 entries: plan_table_lds_kernel and plan_walk_lds_kernel do the
//             table and the write walk with the chunk's nx staged in LDS, a workgroup per chunk)
//  encode  Block::encode (src/block.rs:31-44) + Entry::encode (src/block/builder.rs:72-81) +
//          checksum::calculate_checksum (src/checksum.rs:6-10) + compress::encode Uncompress
//          (src/block/compress.rs:85-89): block b = [u16 n][n x u16 offset][entries][u32 crc]
//          [tag 1] at ext[b] = S(first[b]) + 2 first[b] + 7 b (a closed form: no prefix pass).
//            encode_wave_kernel  one wave per block (payload <= 5104 B, every block_size <= 4 KiB
//                                block): lanes OR their entries into a zeroed LDS window (8-byte
//                                LDS atomics, so entries shorter than a dword need no ownership
//                                rules), the decode's CRC (80-B lane runs, slice-by-16, lane tree)
//                                over the window, then 16-byte stores (the two lines shared with
//                                the neighbouring blocks are written byte-exact)
//            encode_big_kernel   one 16-wave workgroup per longer block (block_size <= 64 KiB):
//                                a wave per entry copies it, 5120-B CRC super-rounds spread over
//                                the waves and shifted to the end with GF(2) multiplies

#include <hip/hip_runtime.h>
#include <cstdlib>
#include <stdint.h>

#include "tpz_internal.h"

namespace tpz {
namespace {

typedef uint32_t u32;
typedef uint64_t u64;
typedef unsigned __int128 u128;

constexpr int kWave = 64;
constexpr int kTableBytes = kNumCrcTables * 256 * 4;  // 41 KiB: the decode's CRC tables

// wave path: 16 waves per CU, each with [guard 96][window 5152] (the window holds A (< 16) +
// payload + crc + tag and the OR spill of the last piece)
constexpr int kEncWaves = 16;
constexpr int kEncThreads = kEncWaves * kWave;
constexpr int kEncGuard = 96;                // zeroed: the CRC's front lane reads <= 79 B before
constexpr int kEncWin = 5152;
constexpr u32 kEncMaxP = 5120 - 16;          // one CRC super-round: A + payload + pad <= 5120
constexpr int kEncSlot = kEncGuard + kEncWin;
static_assert(kTableBytes + kEncWaves * kEncSlot <= 163840, "encode LDS");
static_assert(kEncSlot % 16 == 0 && kTableBytes % 16 == 0, "slot alignment");

// big path: one 16-wave workgroup per block, [tables][guard 96][window][wave CRCs]
constexpr int kBigWaves = 16;
constexpr int kBigThreads = kBigWaves * kWave;
constexpr int kBigWin = 121536;
constexpr u32 kBigMaxP = kBigWin - 48;
constexpr int kBigSuper = (kBigWin + 5119) / 5120;   // CRC super-rounds
static_assert(kTableBytes + kEncGuard + kBigWin + 4 * kBigWaves <= 163840, "big encode LDS");

// ------------------------------------------------------------------ small helpers
// The lane id, laundered: masks and offsets derived from it are recomputed where they are used
// instead of being hoisted out of the block loop into SGPR pairs that spill (tpz_decode.hip).
__device__ __forceinline__ u32 lane_id() {
  u32 l = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  asm volatile("" : "+v"(l));
  return l;
}
__device__ __forceinline__ u32 uni(u32 x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ u32 readlane(u32 x, int l) { return __builtin_amdgcn_readlane(x, l); }
template <int CTRL>
__device__ __forceinline__ u32 dpp(u32 x) {
  return (u32)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, true);
}
constexpr int kRowShl = 0x100;
// Orders one wave's LDS accesses across lanes: the LDS executes a wave's instructions in order,
// so only the compiler has to be kept from moving them.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ u32 be16(u32 x) { return ((x >> 8) & 0xFFu) | ((x & 0xFFu) << 8); }

// ------------------------------------------------------------------ CRC-32 (the decode's tables)
// tab = kNumCrcTables x 256 u32 in LDS: T_0..T_15 (slice-by-16), shift-by-80*2^j operators at
// 16 + 4j, the inverse table at kCrcInvTable (tpz_api.cpp builds them; tpz_decode.hip §CRC).
__device__ __forceinline__ u32 tlook(const u32* tab, int id, u32 byte) { return tab[id * 256 + byte]; }
__device__ __forceinline__ u32 xor3(u32 a, u32 b, u32 c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
__device__ __forceinline__ u32 slice16(const u32* tab, u32 w0, u32 w1, u32 w2, u32 w3) {
  u32 c = xor3(tlook(tab, 15, w0 & 0xFF), tlook(tab, 14, (w0 >> 8) & 0xFF), tlook(tab, 13, (w0 >> 16) & 0xFF));
  c = xor3(c, tlook(tab, 12, w0 >> 24), tlook(tab, 11, w1 & 0xFF));
  c = xor3(c, tlook(tab, 10, (w1 >> 8) & 0xFF), tlook(tab, 9, (w1 >> 16) & 0xFF));
  c = xor3(c, tlook(tab, 8, w1 >> 24), tlook(tab, 7, w2 & 0xFF));
  c = xor3(c, tlook(tab, 6, (w2 >> 8) & 0xFF), tlook(tab, 5, (w2 >> 16) & 0xFF));
  c = xor3(c, tlook(tab, 4, w2 >> 24), tlook(tab, 3, w3 & 0xFF));
  c = xor3(c, tlook(tab, 2, (w3 >> 8) & 0xFF), tlook(tab, 1, (w3 >> 16) & 0xFF));
  return c ^ tlook(tab, 0, w3 >> 24);
}
template <int J>
__device__ __forceinline__ u32 crc_shift(const u32* tab, u32 a) {
  constexpr int b0 = 16 + 4 * J;
  return xor3(tlook(tab, b0, a & 0xFF), tlook(tab, b0 + 1, (a >> 8) & 0xFF),
              tlook(tab, b0 + 2, (a >> 16) & 0xFF)) ^ tlook(tab, b0 + 3, a >> 24);
}
// Un-feed k zero bytes (the inverse of appending them; the top byte of T_0[b] determines b).
__device__ __forceinline__ u32 crc_unshift_small(const u32* tab, u32 r, u32 k) {
  for (u32 i = 0; i < k; i++) {
    const u32 b = tlook(tab, kCrcInvTable, r >> 24);
    r = ((r ^ tlook(tab, 0, b)) << 8) | b;
  }
  return r;
}
// a * b mod P, reflected (bit 31 = x^0): shifts a super-round's CRC to the block end.
__device__ __forceinline__ u32 gf_mul(u32 a, u32 b) {
  u32 p = 0;
#pragma unroll
  for (int i = 0; i < 32; i++) {
    p ^= (a & (0x80000000u >> i)) ? b : 0u;
    b = (b >> 1) ^ ((b & 1u) ? 0xEDB88320u : 0u);
  }
  return p;
}
// The lanes' run CRCs (lane l's run ends 80 l bytes before the end) as one R0: a lane tree of
// shift-by-80*2^k lookups and DPP row shifts (tpz_decode.hip crc_combine).
__device__ __forceinline__ u32 crc_combine(const u32* tab, u32 A) {
  const u32 lane = lane_id();
  if ((lane & 1u) == 1u) A = crc_shift<0>(tab, A);
  A ^= dpp<kRowShl + 1>(A);
  if ((lane & 3u) == 2u) A = crc_shift<1>(tab, A);
  A ^= dpp<kRowShl + 2>(A);
  if ((lane & 7u) == 4u) A = crc_shift<2>(tab, A);
  A ^= dpp<kRowShl + 4>(A);
  if ((lane & 15u) == 8u) A = crc_shift<3>(tab, A);
  A ^= dpp<kRowShl + 8>(A);
  if ((lane & 31u) == 16u) A = crc_shift<4>(tab, A);
  if ((lane & 47u) == 32u) A = crc_shift<5>(tab, A);
  return readlane(A, 0) ^ readlane(A, 16) ^ readlane(A, 32) ^ readlane(A, 48);
}
// R0 of super-round r of the LDS range [pb, pb + Pa) (pb + Pa 16-byte aligned; 5120-B rounds
// counted from the end, 80-B lane runs end-aligned; bytes before pb read from zeroed LDS).
__device__ __forceinline__ u32 round_crc(const u32* tab, const uint8_t* win, int pb, u32 Pa, u32 r) {
  typedef u32 u32x4 __attribute__((ext_vector_type(4)));
  const int seg = (int)Pa - 5120 * (int)r - kCrcLaneBytes * (int)(lane_id() + 1);
  u32 c = 0;
  if (seg + kCrcLaneBytes > 0) {
#pragma unroll
    for (int t = 0; t < kCrcLaneBytes / 16; t++) {
      const u32x4 w = *reinterpret_cast<const u32x4*>(win + pb + seg + 16 * t);
      c = slice16(tab, w.x ^ c, w.y, w.z, w.w);
    }
  }
  return crc_combine(tab, c);
}

// ------------------------------------------------------------------ LDS byte assembly
// The window is zeroed first and every byte is OR-ed in exactly once, so lanes writing bytes of
// one dword need no ordering between them (entries can be 5 bytes long).
__device__ __forceinline__ void lds_or64(uint8_t* W, u32 g, u64 v) {
  __hip_atomic_fetch_or(reinterpret_cast<u64*>(W + g), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_xor64(uint8_t* W, u32 g, u64 v) {
  __hip_atomic_fetch_xor(reinterpret_cast<u64*>(W + g), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// OR the low nb (<= 8) bytes of v into W[d ..)
__device__ __forceinline__ void or_bytes(uint8_t* W, u32 d, u64 v, u32 nb) {
  const u32 g = d & ~7u, sh = d & 7u;
  lds_or64(W, g, v << (8 * sh));
  if (sh + nb > 8) lds_or64(W, g + 8, v >> (64 - 8 * sh));
}
__device__ __forceinline__ void xor_bytes(uint8_t* W, u32 d, u64 v, u32 nb) {
  const u32 g = d & ~7u, sh = d & 7u;
  lds_xor64(W, g, v << (8 * sh));
  if (sh + nb > 8) lds_xor64(W, g + 8, v >> (64 - 8 * sh));
}
// OR 16 bytes (lo, hi) into W[d .. d + 16)
__device__ __forceinline__ void or16(uint8_t* W, u32 d, u64 lo, u64 hi) {
  const u32 g = d & ~7u, sh = d & 7u;
  if (sh == 0) {
    lds_or64(W, g, lo);
    lds_or64(W, g + 8, hi);
  } else {
    lds_or64(W, g, lo << (8 * sh));
    lds_or64(W, g + 8, (lo >> (64 - 8 * sh)) | (hi << (8 * sh)));
    lds_or64(W, g + 16, hi >> (64 - 8 * sh));
  }
}

// 16 bytes of a global buffer of `size` bytes at offset a; bytes past the buffer read as 0.
typedef u128 u128_u __attribute__((aligned(1)));
__device__ __forceinline__ u128 ld16(const uint8_t* base, u64 size, u64 a) {
  if (a + 16 <= size) return *reinterpret_cast<const u128_u*>(base + a);
  u128 v = 0;
  for (u32 i = 0; i < 16 && a + i < size; i++) v |= (u128)base[a + i] << (8 * i);
  return v;
}
__device__ __forceinline__ u128 keep_low(u128 v, u32 m) {   // the low m (<= 16) bytes
  return m >= 16 ? v : (v & (((u128)1 << (8 * m)) - 1));
}
// OR src[0 .. len) (global) into W[d ..): lane-private, 16 bytes per step
__device__ __forceinline__ void copy_in(uint8_t* W, u32 d, const uint8_t* base, u64 size, u64 s,
                                        u32 len) {
  for (u32 t = 0; t < len; t += 16) {
    const u128 v = keep_low(ld16(base, size, s + t), len - t);
    or16(W, d + t, (u64)v, (u64)(v >> 64));
  }
}

// ------------------------------------------------------------------ parameters
struct PlanParams {
  const u64* kpos;
  const u64* vpos;
  u32 n;             // entries
  u32 T;             // block_size - 2: an entry fits while size + encode_len <= T
  u32 span;          // max(1, T / 5): a block holds at most this many entries (each >= 5 B)
  u32* nx;           // n
  u32* info;         // [0] max nx (w), [1] first bad entry (~0u: none): plan_reduce_kernel
  u32* wgmax;        // phase 0: per-workgroup max nx
  u32* wgbad;        // phase 0: per-workgroup first bad entry (~0u: none)
  int* tab_a;        // chunk transfer tables, K x w (w read on the device: info[0])
  int* tab_b;
  u32 C;             // entries per chunk (>= w)
  u32 K;             // chunks
  u32 grid;          // phase 1: workgroups of the grid-stride table / round kernels
  u32* cnt;          // K: blocks per chunk, then their exclusive prefix
  u32* first;        // n + 1: block starts
  u64* ext;          // n + 1: encoded byte extents
  u32* n_blocks;     // one u32
  u32 guess;         // plan_next_kernel: gallop from the mean entry size (0: bisect only)
};

__device__ __forceinline__ u64 S_at(const u64* kpos, const u64* vpos, u64 k0, u64 v0, u32 x) {
  return 4ull * x + (kpos[x] - k0) + (vpos[x] - v0);
}

// ------------------------------------------------------------------ plan kernels
// A workgroup takes kNextPer consecutive entries; the prefix sums its binary searches probe
// (its entries + span) are staged in LDS once. The longest block (w) is reduced per workgroup into
// wgmax[] (a single-address atomic per wave saturated at ~88 per microsecond: 6.4 ms for 2^20
// blocks), then by plan_reduce_kernel.
constexpr u32 kNextWG = 256, kNextPer = kPlanNextPer, kNextTail = 512, kNextWin = kNextPer + kNextTail;

// The window is staged as {kpos, vpos} relative to the workgroup's first entry (u32 pairs: one
// ds_read_b64 per probe, and each entry's own lengths come from LDS too); a window whose bytes do
// not fit u32 takes global probes. A probe sequence starts at the window's mean entry size and
// gallops (4k config: 3 probes per entry instead of 11 for a bisection over span entries).
__global__ __launch_bounds__(kNextWG) void plan_next_kernel(PlanParams p) {
  __shared__ uint2 sw[kNextWin];
  __shared__ u32 wmax[kNextWG / kWave];
  const u32 a0 = blockIdx.x * kNextPer;
  const u64 k0 = p.kpos[a0], v0 = p.vpos[a0];
  // the window: the workgroup's entries and kNextTail more (probes past it read global memory:
  // blocks of more than ~kNextTail / 2 entries); a window of the whole span ahead read 40 % more
  const u32 hiw = (u32)min((u64)p.n, (u64)a0 + kNextWin - 1);   // highest index staged
  const u32 wn = hiw - a0 + 1;
  const bool in_lds = (p.kpos[hiw] - k0) + (p.vpos[hiw] - v0) + 4ull * wn < (1ull << 32);
  if (in_lds) {
    // all of a thread's loads issued before the first LDS write: a loop that stores each pair
    // as it arrives waits out one memory latency per pair
    constexpr u32 kR = kNextWin / kNextWG;
    u64 kk[kR], vv[kR];
#pragma unroll
    for (u32 r = 0; r < kR; r++) {
      const u32 i = threadIdx.x + r * kNextWG;
      if (i < wn) {
        kk[r] = p.kpos[a0 + i];
        vv[r] = p.vpos[a0 + i];
      }
    }
#pragma unroll
    for (u32 r = 0; r < kR; r++) {
      const u32 i = threadIdx.x + r * kNextWG;
      if (i < wn) sw[i] = make_uint2((u32)(kk[r] - k0), (u32)(vv[r] - v0));
    }
  }
  __syncthreads();
  // mean encoded entry size over the window (>= 5 B), rounded up: the gallop's first probe
  const u64 wbytes = 4ull * (wn - 1) + (p.kpos[hiw] - k0) + (p.vpos[hiw] - v0);
  const u64 mean = wn > 1 ? max((u64)5, (wbytes + wn - 2) / (wn - 1)) : 5;
  const bool guess = p.guess;
  u32 mx = 0, bad = ~0u;
  for (u32 a = a0 + threadIdx.x; a < min((u64)p.n, (u64)a0 + kNextPer); a += kNextWG) {
    u64 kl, vl, sa;
    if (in_lds) {
      const uint2 e0 = sw[a - a0], e1 = sw[a + 1 - a0];
      kl = e1.x - e0.x;
      vl = e1.y - e0.y;
      sa = 4ull * (a - a0) + e0.x + e0.y;
    } else {
      kl = p.kpos[a + 1] - p.kpos[a];
      vl = p.vpos[a + 1] - p.vpos[a];
      sa = 4ull * (a - a0) + (p.kpos[a] - k0) + (p.vpos[a] - v0);
    }
    u32 len;
    if (kl == 0 || 4 + kl + vl > p.T) {   // builder.rs:27 assert / an entry no block holds
      bad = min(bad, a);
      len = 1;
    } else {
      const u64 lim = sa + p.T;
      auto S = [&](u32 x) -> u64 {
        if (!in_lds || x - a0 >= wn) return 4ull * (x - a0) + (p.kpos[x] - k0) + (p.vpos[x] - v0);
        const uint2 e = sw[x - a0];
        return 4ull * (x - a0) + e.x + e.y;
      };
      // the block's end b: the largest x in [a + 1, min(n, a + span)] with S(x) <= lim.
      // Invariant: S(lo) <= lim, and hi is past the range or S(hi) > lim (hi itself is never
      // probed while it is the range's exclusive end).
      u32 lo = a + 1, hi = (u32)min((u64)p.n, (u64)a + p.span) + 1;
      if (guess && hi - lo > 1) {   // gallop from the window's mean entry size
        const u32 g = (u32)min((u64)hi - 1, max((u64)lo, (u64)a + p.T / mean));
        if (S(g) <= lim) {
          lo = g;
          u32 d = 1;
          while (d < hi - lo && S(lo + d) <= lim) { lo += d; d <<= 1; }
          if (d < hi - lo) hi = lo + d;
        } else {
          hi = g;
          u32 d = 1;
          while (d < hi - lo && S(hi - d) > lim) { hi -= d; d <<= 1; }
          if (d < hi - lo) lo = hi - d;
        }
      }
      while (hi - lo > 1) {   // then bisect
        const u32 mid = lo + (hi - lo) / 2;
        if (S(mid) <= lim) lo = mid; else hi = mid;
      }
      len = lo - a;
    }
    p.nx[a] = len;
    mx = max(mx, len);
  }
  for (int o = 32; o; o >>= 1) {
    mx = max(mx, (u32)__shfl_xor((int)mx, o));
    bad = min(bad, (u32)__shfl_xor((int)bad, o));
  }
  const u32 lane = lane_id(), wid = threadIdx.x / kWave;
  __shared__ u32 wbad[kNextWG / kWave];
  if (lane == 0) {
    wmax[wid] = mx;
    wbad[wid] = bad;     // ~0u unless the reference rejects an entry
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    u32 m = 0, b = ~0u;
    for (u32 w = 0; w < kNextWG / kWave; w++) {
      m = max(m, wmax[w]);
      b = min(b, wbad[w]);
    }
    p.wgmax[blockIdx.x] = m;
    p.wgbad[blockIdx.x] = b;
  }
}

// info[0] = the longest block in entries (max over wgmax), info[1] = the first entry the reference
// rejects (min over wgbad, ~0u: none); one workgroup. No host initialisation is needed.
__global__ __launch_bounds__(1024) void plan_reduce_kernel(PlanParams p, u32 n_wg) {
  __shared__ u32 part[1024 / kWave], partb[1024 / kWave];
  u32 m = 0, b = ~0u;
  for (u32 i = threadIdx.x; i < n_wg; i += 1024) {
    m = max(m, p.wgmax[i]);
    b = min(b, p.wgbad[i]);
  }
  for (int o = 32; o; o >>= 1) {
    m = max(m, (u32)__shfl_xor((int)m, o));
    b = min(b, (u32)__shfl_xor((int)b, o));
  }
  if (lane_id() == 0) {
    part[threadIdx.x / kWave] = m;
    partb[threadIdx.x / kWave] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (u32 w = 0; w < 1024 / kWave; w++) {
      m = max(m, part[w]);
      b = min(b, partb[w]);
    }
    p.info[0] = m;
    p.info[1] = b;
    p.info[2] = 0;
  }
}

// The longest block in entries, w = info[0] (written by plan_reduce_kernel earlier on the stream):
// the transfer tables' row length. The host sizes them from a bound (span) and the grids stride
// over K x w, so the plan needs no host round trip between its phases.
__device__ __forceinline__ u32 plan_w(const PlanParams& p) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p.info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// tab_a[k w + j] = where the chain entering chunk k at entry k C + j leaves it: the entry
// offset into chunk k + 1, or -1 when it reaches the end of the entries first.
__global__ __launch_bounds__(256) void plan_table_kernel(PlanParams p) {
  const u32 w = plan_w(p);
  const u64 tn = (u64)p.K * w;
  for (u64 t = (u64)blockIdx.x * 256 + threadIdx.x; t < tn; t += (u64)gridDim.x * 256) {
    const u32 k = (u32)(t / w), j = (u32)(t % w);
    const u64 c1 = (u64)(k + 1) * p.C;
    u64 a = (u64)k * p.C + j;
    int F = -1;
    if (a < p.n) {
      const u64 end = min((u64)p.n, c1);
      while (a < end) a += p.nx[a];
      F = a >= p.n ? -1 : (int)(a - c1);
    }
    p.tab_a[t] = F;
  }
}

// One Hillis-Steele round: A_k <- A_k o A_{k-d} (tab_a -> tab_b).
__global__ __launch_bounds__(256) void plan_round_kernel(PlanParams p, u32 d) {
  const u32 w = plan_w(p);
  const u64 tn = (u64)p.K * w;
  for (u64 t = (u64)blockIdx.x * 256 + threadIdx.x; t < tn; t += (u64)gridDim.x * 256) {
    const u32 k = (u32)(t / w), j = (u32)(t % w);
    int v = p.tab_a[t];
    if (k >= d) {
      const int x = p.tab_a[(u64)(k - d) * w + j];
      v = x < 0 ? -1 : p.tab_a[(u64)k * w + x];
    }
    p.tab_b[t] = v;
  }
}

// The chain's entry into chunk k (absolute entry index), or ~0u if it ended before.
__device__ __forceinline__ u64 chunk_entry(const PlanParams& p, u32 k) {
  if (k == 0) return 0;
  const int e = p.tab_a[(u64)(k - 1) * plan_w(p)];
  return e < 0 ? ~0ull : (u64)k * p.C + (u32)e;
}

__global__ __launch_bounds__(256) void plan_count_kernel(PlanParams p) {
  const u32 k = blockIdx.x * 256 + threadIdx.x;
  if (k >= p.K) return;
  u64 a = chunk_entry(p, k);
  u32 c = 0;
  if (a != ~0ull) {
    const u64 end = min((u64)p.n, (u64)(k + 1) * p.C);
    for (; a < end; a += p.nx[a]) c++;
  }
  p.cnt[k] = c;
}

// Exclusive prefix of cnt in place (one workgroup); the total goes to *n_blocks.
__global__ __launch_bounds__(1024) void plan_scan_kernel(PlanParams p) {
  __shared__ u32 part[1024 / kWave];
  __shared__ u32 carry_s;
  if (threadIdx.x == 0) carry_s = 0;
  __syncthreads();
  const u32 lane = lane_id(), wid = threadIdx.x / kWave;
  for (u32 base = 0; base < p.K; base += 1024) {
    const u32 k = base + threadIdx.x;
    const u32 v = k < p.K ? p.cnt[k] : 0u;
    u32 x = v;                                   // inclusive wave scan
    for (int o = 1; o < kWave; o <<= 1) {
      const u32 y = (u32)__shfl_up((int)x, o);
      if (lane >= (u32)o) x += y;
    }
    if (lane == kWave - 1) part[wid] = x;
    __syncthreads();
    u32 before = carry_s;
    for (u32 w = 0; w < wid; w++) before += part[w];
    if (k < p.K) p.cnt[k] = before + x - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry_s = before + x;
    __syncthreads();
  }
  if (threadIdx.x == 0) *p.n_blocks = carry_s;
}

__global__ __launch_bounds__(256) void plan_write_kernel(PlanParams p) {
  const u32 k = blockIdx.x * 256 + threadIdx.x;
  if (k >= p.K) return;
  const u64 k0 = p.kpos[0], v0 = p.vpos[0];
  u64 a = chunk_entry(p, k);
  u32 b = p.cnt[k];
  if (a != ~0ull) {
    const u64 end = min((u64)p.n, (u64)(k + 1) * p.C);
    for (; a < end; a += p.nx[a], b++) {
      p.first[b] = (u32)a;
      p.ext[b] = S_at(p.kpos, p.vpos, k0, v0, (u32)a) + 2 * a + 7ull * b;   // SsTableBuilder data.len()
    }
  }
  if (k + 1 == p.K) {
    const u32 nb = *p.n_blocks;
    p.first[nb] = p.n;
    p.ext[nb] = S_at(p.kpos, p.vpos, k0, v0, p.n) + 2ull * p.n + 7ull * nb;
  }
}

// The table and the write walk with the chunk's nx staged in LDS (chunks of <= kWalkMaxC entries):
// a step is an LDS read instead of a dependent global load, and the write kernel no longer waits
// on its own first/ext stores between steps (vmcnt counts stores too). One workgroup per chunk.
constexpr u32 kWalkMaxC = 8192;

__device__ __forceinline__ u32 stage_chunk_nx(const PlanParams& p, u32 k, u32* snx) {
  const u64 c0 = (u64)k * p.C;
  const u32 len = (u32)(min((u64)p.n, c0 + p.C) - c0);
  // eight loads in flight per thread before their LDS writes (one latency per eight words)
  for (u32 i0 = threadIdx.x; i0 < len; i0 += 8 * blockDim.x) {
    u32 v[8];
#pragma unroll
    for (u32 r = 0; r < 8; r++) {
      const u32 i = i0 + r * blockDim.x;
      if (i < len) v[r] = p.nx[c0 + i];
    }
#pragma unroll
    for (u32 r = 0; r < 8; r++) {
      const u32 i = i0 + r * blockDim.x;
      if (i < len) snx[i] = v[r];
    }
  }
  __syncthreads();
  return len;
}

__global__ __launch_bounds__(256) void plan_table_lds_kernel(PlanParams p) {
  extern __shared__ u32 snx[];
  const u32 k = blockIdx.x;
  const u32 len = stage_chunk_nx(p, k, snx);
  const u32 w = plan_w(p);
  for (u32 j = threadIdx.x; j < w; j += blockDim.x) {
    int F = -1;
    if (j < len) {
      u32 r = j;
      while (r < len) r += snx[r];
      const u64 a = (u64)k * p.C + r;
      F = a >= p.n ? -1 : (int)(r - p.C);
    }
    p.tab_a[(u64)k * w + j] = F;
  }
}

__global__ __launch_bounds__(256) void plan_walk_lds_kernel(PlanParams p) {
  extern __shared__ u32 snx[];
  uint16_t* st = reinterpret_cast<uint16_t*>(snx + p.C);     // the chunk's block starts, chunk-relative
  __shared__ u32 s_count;
  const u32 k = blockIdx.x;
  const u64 c0 = (u64)k * p.C;
  const u32 len = stage_chunk_nx(p, k, snx);
  if (threadIdx.x == 0) {
    const u64 a = chunk_entry(p, k);
    u32 c = 0;
    if (a != ~0ull)
      for (u32 r = (u32)(a - c0); r < len; r += snx[r]) st[c++] = (uint16_t)r;
    s_count = c;
  }
  __syncthreads();
  const u32 c = s_count;
  const u64 k0 = p.kpos[0], v0 = p.vpos[0];
  const u32 b0 = p.cnt[k];
  for (u32 i = threadIdx.x; i < c; i += blockDim.x) {
    const u32 a = (u32)(c0 + st[i]);
    const u64 b = (u64)b0 + i;
    p.first[b] = a;
    p.ext[b] = S_at(p.kpos, p.vpos, k0, v0, a) + 2ull * a + 7ull * b;   // SsTableBuilder data.len()
  }
  if (k + 1 == p.K && threadIdx.x == 0) {
    const u32 nb = *p.n_blocks;
    p.first[nb] = p.n;
    p.ext[nb] = S_at(p.kpos, p.vpos, k0, v0, p.n) + 2ull * p.n + 7ull * nb;
  }
}

// ------------------------------------------------------------------ encode kernels
struct EncParams {
  const uint8_t* keys;
  const u64* kpos;
  u64 key_bytes;     // readable bytes of keys (kpos[n])
  const uint8_t* vals;
  const u64* vpos;
  u64 val_bytes;
  const u32* first;  // n_blocks + 1
  const u64* ext;    // n_blocks + 1
  u32 n_blocks;
  const u32* plan_info;      // non-null: tpz_plan_blocks_async's {w, bad entry, n_blocks} on the device
  const u32* crc_tables;
  uint8_t* out;      // 16-byte aligned
  u32* big_list;     // workspace: blocks for encode_big_kernel
  u32* big_count;    // zeroed before the launch
  u32 xp[kBigSuper]; // x^(8 * 5120 r) mod P: super-round r's shift to the block end
};

// Stores W[A, A + len) to out[o0, o0 + len) (o0 & 15 == A): whole 16-byte pieces for the lines
// inside the block, byte-exact stores for the pieces it shares with its neighbours.
__device__ __forceinline__ void store_block(const uint8_t* W, uint8_t* out, u64 o0, u32 A, u32 len,
                                            u32 t0, u32 nt) {
  const u32 end = A + len, npieces = (end + 15) / 16;
  uint8_t* g = out + (o0 & ~15ull);
  for (u32 q = t0; q < npieces; q += nt) {
    const bool edge = (q == 0 && A != 0) || (q + 1 == npieces && (end & 15u) != 0);
    const uint4 v = *reinterpret_cast<const uint4*>(W + 16 * q);
    if (!edge) {
      *reinterpret_cast<uint4*>(g + 16 * q) = v;
    } else {
      const u32 lo = q == 0 ? A : 0u, hi = min(16u, end - 16 * q);
      for (u32 i = lo; i < hi; i++) g[16 * q + i] = W[16 * q + i];
    }
  }
}

// One block's entries: n (BE u16), the offsets and Entry::encode of each entry, OR-ed into W.
// Threads t0, t0 + nt, ... take the offsets; entry copies go per thread (wave path).
__device__ __forceinline__ void put_offsets(const EncParams& p, uint8_t* W, u32 A, u32 a, u32 nb,
                                            u64 kp0, u64 vp0, u32 t0, u32 nt) {
  for (u32 i = t0; i < nb; i += nt) {
    const u32 x = a + i;
    const u64 off = 4ull * i + (p.kpos[x] - kp0) + (p.vpos[x] - vp0);
    or_bytes(W, A + 2 + 2 * i, be16((u32)off & 0xFFFFu), 2);   // builder.rs:37 (size as u16)
  }
}

constexpr int kEncLds = kTableBytes + kEncWaves * kEncSlot;
constexpr int kBigEncLds = kTableBytes + kEncGuard + kBigWin + 4 * kBigWaves;

// The wave path keeps three blocks in flight per wave: block i is assembled from pieces loaded
// during block i - 1, the pieces of block i + 1 are issued as soon as block i's are in LDS (their
// kpos/vpos arrived during block i - 1), and block i + 2's kpos/vpos are issued at the start of
// block i; the blocks' first/ext come 64 blocks at a time (lane l: the wave's block g*64 + l).
constexpr int kPre = 8;                      // prefetched 16-B pieces per lane (key, then value)

// The lengths are taken from the raw next offsets where they are used (a block after the
// load): subtracting at the load made the wave wait for it, and for everything issued before it
// (the previous block's stores), at the start of every block.
struct EntryRegs {                           // the lane's entry in a block's first 64
  u64 kp, vp;                                // kpos[x], vpos[x]
  u32 k1, v1;                                // low words of kpos[x + 1], vpos[x + 1]
  __device__ __forceinline__ u32 kl() const { return k1 - (u32)kp; }   // < 2^16 in any block
  __device__ __forceinline__ u32 vl() const { return v1 - (u32)vp; }
};

__device__ __forceinline__ EntryRegs load_entry(const EncParams& p, u32 a, u32 e, bool live) {
  const u32 x = a + lane_id();
  EntryRegs r{0, 0, 0, 0};
  if (live && x < e) {
    r.kp = p.kpos[x];
    r.k1 = (u32)p.kpos[x + 1];
    r.vp = p.vpos[x];
    r.v1 = (u32)p.vpos[x + 1];
  }
  return r;
}

// piece k of the lane's entry: key pieces (nk of them), then value pieces
__device__ __forceinline__ u128 load_piece(const EncParams& p, const EntryRegs& r, u32 nk, u32 k) {
  return k < nk ? ld16(p.keys, p.key_bytes, r.kp + 16ull * k)
                : ld16(p.vals, p.val_bytes, r.vp + 16ull * (k - nk));
}

__device__ __forceinline__ void issue_pieces(const EncParams& p, const EntryRegs& r, u128 (&pf)[kPre]) {
  const u32 nk = (r.kl() + 15) / 16, nt = nk + (r.vl() + 15) / 16;
#pragma unroll
  for (int k = 0; k < kPre; k++) pf[k] = (u32)k < nt ? load_piece(p, r, nk, k) : (u128)0;
}

// OR piece k (value v) of an entry whose klen field sits at W[pos] into the window
__device__ __forceinline__ void emit_piece(uint8_t* W, u32 pos, u64 kl, u64 vl, u32 nk, u32 k, u128 v) {
#ifdef TPZ_ENC_ABL_NOASM   // diagnostic (timing only, wrong bytes): the pieces are loaded, not placed
  asm volatile("" ::"v"((u32)v), "v"((u32)(v >> 32)), "v"((u32)(v >> 64)), "v"((u32)(v >> 96)));
  return;
#endif
  const bool key = k < nk;
  const u32 j = key ? k : k - nk;
  const u32 rem = (u32)((key ? kl : vl) - 16ull * j);
  v = keep_low(v, rem);
  or16(W, pos + (key ? 2u : 4u + (u32)kl) + 16 * j, (u64)v, (u64)(v >> 64));
}

struct BlockMeta {
  u32 a, e;
  u64 o0, o1;
};

__global__ __launch_bounds__(kEncThreads) void encode_wave_kernel(EncParams p) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kEncLds];
  u32* tab = reinterpret_cast<u32*>(lds);
  const u32 lane = lane_id(), wid = threadIdx.x / kWave;
  uint8_t* slot = lds + kTableBytes + wid * kEncSlot;
  uint8_t* W = slot + kEncGuard;
  for (int i = threadIdx.x; i < kTableBytes / 16; i += kEncThreads)
    reinterpret_cast<uint4*>(lds)[i] = reinterpret_cast<const uint4*>(p.crc_tables)[i];
  for (int i = lane; i < kEncGuard / 16; i += kWave) reinterpret_cast<uint4*>(slot)[i] = make_uint4(0, 0, 0, 0);
  __shared__ u32 chunk_next;          // the workgroup's next unclaimed chunk
  if (threadIdx.x == 0) chunk_next = 0;
  __syncthreads();

  const u32 nwaves = gridDim.x * kEncWaves;
  // a plan with a rejected entry (tpz_plan_blocks_async) encodes nothing
  const u32 n_blocks = !p.plan_info ? p.n_blocks : (uni(p.plan_info[1]) != ~0u ? 0u : uni(p.plan_info[2]));
  // The workgroup's blocks are the rows r nwaves + kEncWaves blockIdx.x + [0, kEncWaves), in
  // chunks of kEncChunk; a wave takes the next chunk from an LDS counter when it finishes one
  // (the waves of a CU do not run at one speed: the decode's wave path, tpz_decode.hip). Lane l
  // of a chunk's group holds first[] / ext[] of the chunk's block l.
#ifndef TPZ_ENC_CHUNK
#define TPZ_ENC_CHUNK 4
#endif
  constexpr u32 kEncChunk = TPZ_ENC_CHUNK, kPerRow = kEncWaves / kEncChunk;
  static_assert(kEncWaves % kEncChunk == 0 && kEncChunk >= 2, "block i + 2 is in the next chunk at most");
  const u32 row0 = blockIdx.x * kEncWaves;
  auto chunk_first = [&](u32 q) -> u32 {
    const u64 f = (u64)(q / kPerRow) * nwaves + row0 + (q % kPerRow) * kEncChunk;
    return f < n_blocks ? (u32)f : n_blocks;
  };
  auto claim_chunk = [&]() -> u32 {
    u32 q = 0;
    if (lane == 0) q = atomicAdd(&chunk_next, 1u);
    return uni(q);
  };
  // every lane loads (indices clamped to the table, whose n_blocks + 1 entries exist): a masked
  // load merged into the old registers made the wave wait for it as soon as it was issued
  auto load_group = [&](u32 q, BlockMeta& m) {
    const u32 cf = chunk_first(q);
    const u32 b = min(cf + min(lane, kEncChunk - 1), n_blocks), b1 = min(b + 1, n_blocks);
    m.a = p.first[b];
    m.e = p.first[b1];
    m.o0 = p.ext[b];
    m.o1 = p.ext[b1];
  };
  auto pick = [&](const BlockMeta& m, u32 l) {
    BlockMeta r;
    r.a = readlane(m.a, (int)l);
    r.e = readlane(m.e, (int)l);
    r.o0 = ((u64)readlane((u32)(m.o0 >> 32), (int)l) << 32) | readlane((u32)m.o0, (int)l);
    r.o1 = ((u64)readlane((u32)(m.o1 >> 32), (int)l) << 32) | readlane((u32)m.o1, (int)l);
    return r;
  };
  if (n_blocks == 0) return;
  BlockMeta gA{0, 0, 0, 0}, gB{0, 0, 0, 0};                 // chunks qa and qb
  u32 qa = claim_chunk(), qb = claim_chunk();
  load_group(qa, gA);
  load_group(qb, gB);
  u32 fa = chunk_first(qa), fb = chunk_first(qb);
  // block t of the wave's two chunks (t < 2 kEncChunk): its index (n_blocks: none) and meta
  auto block_of = [&](u32 t) -> u32 {
    const u32 bb = t < kEncChunk ? fa + t : fb + (t - kEncChunk);
    return bb < n_blocks ? bb : n_blocks;
  };
  auto meta_of = [&](u32 t) { return t < kEncChunk ? pick(gA, t) : pick(gB, t - kEncChunk); };
  if (block_of(0) >= n_blocks) return;

  const bool has1 = block_of(1) < n_blocks;
  BlockMeta m0 = meta_of(0), m1 = meta_of(has1 ? 1 : 0);
  EntryRegs cur = load_entry(p, m0.a, m0.e, true);
  EntryRegs nxt = load_entry(p, m1.a, m1.e, has1);
  u128 pf[kPre];
  issue_pieces(p, cur, pf);

#ifdef TPZ_ENC_ABL_ROTPRIO   // diagnostic: rotate the wave's issue priority every block
  u32 rot = blockIdx.x * kEncWaves + wid;
#endif
  for (u32 j = 0;;) {                                        // block j of chunk qa
    const u32 b = block_of(j);
    if (b >= n_blocks) break;
#ifdef TPZ_ENC_ABL_ROTPRIO
    switch (uni(rot++) & 3u) {
      case 0: __builtin_amdgcn_s_setprio(0); break;
      case 1: __builtin_amdgcn_s_setprio(1); break;
      case 2: __builtin_amdgcn_s_setprio(2); break;
      default: __builtin_amdgcn_s_setprio(3); break;
    }
#endif
    const BlockMeta m = meta_of(j);

    const u32 a = m.a, nb = m.e - m.a;
    const u64 o0 = m.o0;
    const u32 A = (u32)(o0 & 15);
    const u32 P = (u32)(m.o1 - o0 - 5);
    const bool small = P + A <= kEncMaxP;
    if (small) {
      const u32 zn = (A + P + 5 + 24 + 15) / 16;
      for (u32 q = lane; q < zn; q += kWave) reinterpret_cast<uint4*>(W)[q] = make_uint4(0, 0, 0, 0);
      wave_sync();
      const u64 kp0 = ((u64)readlane((u32)(cur.kp >> 32), 0) << 32) | readlane((u32)cur.kp, 0);
      const u64 vp0 = ((u64)readlane((u32)(cur.vp >> 32), 0) << 32) | readlane((u32)cur.vp, 0);
      if (lane == 0) or_bytes(W, A, be16(nb & 0xFFFFu), 2);         // block.rs:35 (n as u16)
      {                                                              // entries 0..63 from registers
        const u64 kl = cur.kl(), vl = cur.vl();
        if (lane < nb) {
          const u64 off = 4ull * lane + (cur.kp - kp0) + (cur.vp - vp0);
          or_bytes(W, A + 2 + 2 * lane, be16((u32)off & 0xFFFFu), 2);   // builder.rs:37
          const u32 pos = A + 2 + 2 * nb + (u32)off;
          or_bytes(W, pos, be16((u32)kl & 0xFFFFu), 2);               // Entry::encode
          or_bytes(W, pos + 2 + (u32)kl, be16((u32)vl & 0xFFFFu), 2);
          const u32 nk = (u32)((kl + 15) / 16), nt = nk + (u32)((vl + 15) / 16);
#pragma unroll
          for (int k = 0; k < kPre; k++)
            if ((u32)k < nt) emit_piece(W, pos, kl, vl, nk, k, pf[k]);
          for (u32 k = kPre; k < nt; k++) emit_piece(W, pos, kl, vl, nk, k, load_piece(p, cur, nk, k));
        }
      }
      if (nb > kWave) {                                              // entries 64.. (tiny entries)
        put_offsets(p, W, A, a, nb, kp0, vp0, kWave + lane, kWave);
        for (u32 i2 = kWave + lane; i2 < nb; i2 += kWave) {
          const u32 x = a + i2;
          const u64 kp = p.kpos[x], kl = p.kpos[x + 1] - kp, vp = p.vpos[x], vl = p.vpos[x + 1] - vp;
          const u32 pos = A + 2 + 2 * nb + (u32)(4ull * i2 + (kp - kp0) + (vp - vp0));
          or_bytes(W, pos, be16((u32)kl & 0xFFFFu), 2);
          copy_in(W, pos + 2, p.keys, p.key_bytes, kp, (u32)kl);
          or_bytes(W, pos + 2 + (u32)kl, be16((u32)vl & 0xFFFFu), 2);
          copy_in(W, pos + 4 + (u32)kl, p.vals, p.val_bytes, vp, (u32)vl);
        }
      }
    } else {                                                         // longer block: big kernel
      if (lane == 0) p.big_list[atomicAdd(p.big_count, 1u)] = b;
    }
    // (the pieces are issued from one site: with a copy per branch the array was merged at the
    // end of the iteration, a register copy that waited for the loads just issued)
    wave_sync();
    // block i + 2's kpos / vpos and block i + 1's pieces, issued after the block's first wait
    // for its own registers (which, issued earlier, also waited for these)
    const bool has2 = block_of(j + 2) < n_blocks;
    const BlockMeta m2 = meta_of(has2 ? j + 2 : j);
    const EntryRegs nn = load_entry(p, m2.a, m2.e, has2);
    issue_pieces(p, nxt, pf);
    if (small) {
      const u32 kpad = (16 - ((A + P) & 15)) & 15;       // zero bytes up to the 16-byte boundary
      // checksum::calculate_checksum over the payload: init 0xFFFFFFFF folded into its first
      // four bytes, raw CRC of payload || 0^kpad, un-shifted, complemented
      if (lane == 0) xor_bytes(W, A, 0xFFFFFFFFull, 4);
      wave_sync();
#ifdef TPZ_ENC_ABL_NOCRC   // diagnostic (timing only, wrong CRCs)
      const u32 R = kpad;
#else
      const u32 R = round_crc(tab, slot, kEncGuard + (int)A, P + kpad, 0);
#endif
      wave_sync();
      const u32 crc = ~crc_unshift_small(tab, R, kpad);
      if (lane == 0) {
        xor_bytes(W, A, 0xFFFFFFFFull, 4);
        or_bytes(W, A + P, __builtin_bswap32(crc), 4);               // block.rs:42 (put_u32, BE)
        or_bytes(W, A + P + 4, 1, 1);                                 // compress.rs:87 tag
      }
      wave_sync();
#ifndef TPZ_ENC_ABL_NOSTORE   // diagnostic (timing only): nothing written
      store_block(W, p.out, o0, A, P + 5, lane, kWave);
#endif
      wave_sync();
    }
    cur = nxt;
    nxt = nn;
    if (++j == kEncChunk) {          // next chunk (its meta loaded a chunk ago)
      j = 0;
      qa = qb;
      fa = fb;
      gA = gB;
      // the copy is made before the next loads are issued, so that they land in gB's registers
      // (not in temporaries copied over as soon as they are issued, which waited for them)
      asm volatile("" : "+v"(gA.a), "+v"(gA.e), "+v"(gA.o0), "+v"(gA.o1)::"memory");
      qb = claim_chunk();
      fb = chunk_first(qb);
      load_group(qb, gB);
    }
  }
}

__global__ __launch_bounds__(kBigThreads) void encode_big_kernel(EncParams p) {
  const u32 cnt = uni(*p.big_count);
  if (cnt == 0) return;                                  // before loading the tables
  __shared__ __attribute__((aligned(16))) uint8_t lds[kBigEncLds];
  u32* tab = reinterpret_cast<u32*>(lds);
  uint8_t* slot = lds + kTableBytes;
  uint8_t* W = slot + kEncGuard;
  u32* wcrc = reinterpret_cast<u32*>(W + kBigWin);
  const u32 lane = lane_id(), wid = threadIdx.x / kWave;
  for (int i = threadIdx.x; i < kTableBytes / 16; i += kBigThreads)
    reinterpret_cast<uint4*>(lds)[i] = reinterpret_cast<const uint4*>(p.crc_tables)[i];
  for (int i = threadIdx.x; i < kEncGuard / 16; i += kBigThreads) reinterpret_cast<uint4*>(slot)[i] = make_uint4(0, 0, 0, 0);
  for (u32 it = blockIdx.x; it < cnt; it += gridDim.x) {
    const u32 b = p.big_list[it];
    const u32 a = p.first[b], e = p.first[b + 1], nb = e - a;
    const u64 o0 = p.ext[b], len = p.ext[b + 1] - o0;
    const u32 A = (u32)(o0 & 15);
    const u32 P = (u32)(len - 5);
    if (P + A > kBigMaxP) continue;                      // rejected by tpz_plan_blocks (block_size)
    const u32 kpad = (16 - ((A + P) & 15)) & 15;
    const u32 zn = (A + P + 5 + 24 + 15) / 16;
    __syncthreads();                                     // the previous block's store read W
    for (u32 q = threadIdx.x; q < zn; q += kBigThreads) reinterpret_cast<uint4*>(W)[q] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    const u64 kp0 = p.kpos[a], vp0 = p.vpos[a];
    if (threadIdx.x == 0) or_bytes(W, A, be16(nb & 0xFFFFu), 2);
    put_offsets(p, W, A, a, nb, kp0, vp0, threadIdx.x, kBigThreads);
    for (u32 i = wid; i < nb; i += kBigWaves) {          // one wave per entry, 16-B pieces per lane
      const u32 x = a + i;
      const u64 kp = p.kpos[x], kl = p.kpos[x + 1] - kp, vp = p.vpos[x], vl = p.vpos[x + 1] - vp;
      const u32 pos = A + 2 + 2 * nb + (u32)(4ull * i + (kp - kp0) + (vp - vp0));
      if (lane == 0) {
        or_bytes(W, pos, be16((u32)kl & 0xFFFFu), 2);
        or_bytes(W, pos + 2 + (u32)kl, be16((u32)vl & 0xFFFFu), 2);
      }
      for (u32 t = 16 * lane; t < kl; t += 16 * kWave) {
        const u128 v = keep_low(ld16(p.keys, p.key_bytes, kp + t), (u32)kl - t);
        or16(W, pos + 2 + t, (u64)v, (u64)(v >> 64));
      }
      for (u32 t = 16 * lane; t < vl; t += 16 * kWave) {
        const u128 v = keep_low(ld16(p.vals, p.val_bytes, vp + t), (u32)vl - t);
        or16(W, pos + 4 + (u32)kl + t, (u64)v, (u64)(v >> 64));
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) xor_bytes(W, A, 0xFFFFFFFFull, 4);
    __syncthreads();
    const u32 Pa = P + kpad, Sr = (Pa + 5119) / 5120;
    u32 acc = 0;
    for (u32 r = wid; r < Sr; r += kBigWaves) acc ^= gf_mul(p.xp[r], round_crc(tab, slot, kEncGuard + (int)A, Pa, r));
    if (lane == 0) wcrc[wid] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      u32 R = 0;
      for (int w = 0; w < kBigWaves; w++) R ^= wcrc[w];
      const u32 crc = ~crc_unshift_small(tab, R, kpad);
      xor_bytes(W, A, 0xFFFFFFFFull, 4);
      or_bytes(W, A + P, __builtin_bswap32(crc), 4);
      or_bytes(W, A + P + 4, 1, 1);
    }
    __syncthreads();
    store_block(W, p.out, o0, A, P + 5, threadIdx.x, kBigThreads);
  }
}

// ------------------------------------------------------------------ host side
u32 gf_mul_host(u32 a, u32 b) {
  u32 p = 0;
  for (int i = 0; i < 32; i++) {
    if (a & (0x80000000u >> i)) p ^= b;
    b = (b >> 1) ^ ((b & 1u) ? 0xEDB88320u : 0u);
  }
  return p;
}
u32 x8n_host(u64 n) {                    // x^(8n) mod P, reflected
  u32 r = 0x80000000u, sq = 0x00800000u;  // x^0, x^8
  for (; n; n >>= 1) {
    if (n & 1u) r = gf_mul_host(r, sq);
    sq = gf_mul_host(sq, sq);
  }
  return r;
}

}  // namespace

hipError_t launch_plan(const PlanLaunch& a, hipStream_t s) {
  PlanParams p{};
  p.kpos = a.kpos;
  p.vpos = a.vpos;
  p.n = a.n;
  p.T = a.block_size - 2;
  p.span = p.T / 5 ? p.T / 5 : 1;
  p.nx = a.nx;
  p.info = a.info;
  p.first = a.first;
  p.ext = a.ext;
  p.n_blocks = a.n_blocks;
  p.cnt = a.cnt;
  p.C = a.chunk ? a.chunk : 1;
  p.K = (u32)(((u64)a.n + p.C - 1) / p.C);
  hipError_t e;
  if (a.phase == 0) {
    const u32 nwg = (u32)(((u64)a.n + kNextPer - 1) / kNextPer);
    p.wgmax = a.nx + a.n;                 // the caller sizes nx for n + 2 (n / 2048 + 1) words
    p.wgbad = p.wgmax + nwg;
    static const bool bisect = std::getenv("TPZ_PLAN_BISECT") != nullptr;   // A/B probe
    p.guess = bisect ? 0u : 1u;
    plan_next_kernel<<<nwg, kNextWG, 0, s>>>(p);
    plan_reduce_kernel<<<1, 1024, 0, s>>>(p, nwg);
    return hipGetLastError();
  }
  // grid-stride table / round kernels over K x w (w on the device; a.w is its bound)
  const u64 tn = (u64)p.K * a.w;
  const u64 tg_full = (tn + 255) / 256;
  const u32 tg = (u32)(tg_full < 2048 ? (tg_full ? tg_full : 1) : 2048);
  p.grid = tg;
  p.tab_a = a.tab_a;
  p.tab_b = a.tab_b;
  static const bool global_walk = std::getenv("TPZ_PLAN_GLOBAL_WALK") != nullptr;   // A/B probe
  const bool lds = p.C <= kWalkMaxC && !global_walk;
  if (lds)
    plan_table_lds_kernel<<<p.K, 256, p.C * 4, s>>>(p);
  else
    plan_table_kernel<<<tg, 256, 0, s>>>(p);
  for (u32 d = 1; d < p.K; d <<= 1) {
    plan_round_kernel<<<tg, 256, 0, s>>>(p, d);
    int* t = p.tab_a;
    p.tab_a = p.tab_b;
    p.tab_b = t;
  }
  const u32 kg = (p.K + 255) / 256;
  if (lds) {   // the count walk stays in global memory: it has no stores to wait on and touches
               // only the chain's own nx lines (33 us against 45 us staged, 4k shard)
    plan_count_kernel<<<kg, 256, 0, s>>>(p);
    plan_scan_kernel<<<1, 1024, 0, s>>>(p);
    plan_walk_lds_kernel<<<p.K, 256, p.C * 6, s>>>(p);
  } else {
    plan_count_kernel<<<kg, 256, 0, s>>>(p);
    plan_scan_kernel<<<1, 1024, 0, s>>>(p);
    plan_write_kernel<<<kg, 256, 0, s>>>(p);
  }
  e = hipGetLastError();
  return e;
}

hipError_t launch_encode(const EncodeLaunch& a, hipStream_t s) {
  EncParams p{};
  p.keys = a.keys;
  p.kpos = a.kpos;
  p.key_bytes = a.key_bytes;
  p.vals = a.vals;
  p.vpos = a.vpos;
  p.val_bytes = a.val_bytes;
  p.first = a.first;
  p.ext = a.ext;
  p.n_blocks = a.n_blocks;
  p.plan_info = a.plan_info;
  p.crc_tables = a.crc_tables;
  p.out = a.out;
  p.big_list = a.big_list;
  p.big_count = a.big_count;
  for (int r = 0; r < kBigSuper; r++) p.xp[r] = x8n_host(5120ull * r);
  hipError_t e = hipMemsetAsync(a.big_count, 0, 4, s);
  if (e != hipSuccess) return e;
  const u32 grid = a.num_cus;
  encode_wave_kernel<<<grid, kEncThreads, 0, s>>>(p);
  encode_big_kernel<<<grid, kBigThreads, 0, s>>>(p);
  return hipGetLastError();
}

u32 encode_max_payload() { return kBigMaxP; }

}  // namespace tpz
