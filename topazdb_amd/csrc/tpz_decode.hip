// tpz_decode.hip — gfx950 kernels for topazdb's SSTable block decode + CRC-32 verify.
//
// Restates, on the device, for every block of a batch:
//   compress::decode tag dispatch          src/block/compress.rs:95-113
//   Block::decode (crc split, n, offsets)  src/block.rs:46-65
//   checksum::verify_checksum (crc32fast)  src/checksum.rs:6-21
//   BlockIterator::seek_to for every entry src/block/iterator.rs:63-83
// into the slotted column layout of include/tpz_gpu.h.
//
// Execution model:
//  * wave path  — one 64-lane wave owns one block at a time; 16 waves per 1024-thread
//    workgroup, one workgroup per CU, persistent over the batch. The NEXT block's bytes are
//    prefetched into VGPRs (5 x dwordx4 per lane = 5 KiB per wave) while the current block is
//    processed out of the wave's LDS slot, so HBM reads stay in flight during the decode.
//  * big path   — blocks that do not fit a wave slot (len > 5104 B or n > 256) are appended to
//    a device worklist by the wave path and decoded by a second kernel, one wave per block with
//    a 92 KiB LDS window (TPZ_MAX_BLOCK_BYTES: every block a 64 KiB-target BlockBuilder can
//    emit) and its entry table in a per-workgroup global scratch (no entry-count limit).
//  CRC-32: payload split into 16-byte chunks aligned to the payload END; lane l folds chunks
//  l, l+64, ... (Horner with a shift-by-1024 operator), then a 6-level lane tree combines with
//  shift-by-16*2^k operators. All operators are byte-sliced lookup tables in LDS (40 KiB).
//  Decode: lanes parse 64 entries at a time (n, offsets, klen, vlen, bounds checks that mirror
//  the reference's panics), a wave prefix sum gives packed output positions, then each lane
//  assembles 16-byte output chunks (output-driven gather, coalesced 1 KiB dwordx4 stores).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tpz_internal.h"

namespace tpz {

typedef uint32_t u32;
typedef uint64_t u64;

// ------------------------------------------------------------------ LDS geometry
constexpr int kWave = 64;
constexpr int kWavesPerWG = 16;
constexpr int kWGThreads = kWave * kWavesPerWG;
constexpr int kTableBytes = kNumCrcTables * 256 * 4;  // 40 KiB
constexpr int kGuard = 32;

// wave path slot: [guard 32][window 5120][pad 32][ktab 256 x u32][vtab 256 x u32]
constexpr int kWinRounds = 5;                       // 5 x 1 KiB window
constexpr int kWinBytes = kWinRounds * 1024;
constexpr u32 kWaveMaxLen = kWinBytes - 16;         // a0 (<=15) + len must fit the window
constexpr u32 kWaveMaxN = 256;
constexpr int kSlotBytes = kGuard + kWinBytes + 32 + kWaveMaxN * 8;
static_assert(kSlotBytes % 16 == 0, "slot alignment");
constexpr int kWaveLds = kTableBytes + kWavesPerWG * kSlotBytes;
static_assert(kWaveLds <= 163840, "wave path LDS");

// big path (one wave per block): [guard][window 92 KiB][pad]; entry table in global scratch
constexpr int kBigWinBytes = 94208;
constexpr u32 kBigMaxLen = TPZ_MAX_BLOCK_BYTES;     // 94192 (a0 + len <= window)
constexpr int kBigLds = kTableBytes + kGuard + kBigWinBytes + 32;
static_assert(kBigMaxLen + 16 <= kBigWinBytes, "big window");
static_assert(kBigLds <= 163840, "big path LDS");

constexpr uint8_t kStDeferred = 0xFF;  // internal: handed to the big path

// ------------------------------------------------------------------ small helpers
__device__ __forceinline__ u32 lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ u32 uni(u32 x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ u64 uni64(u64 x) {
  u32 lo = __builtin_amdgcn_readfirstlane((u32)x), hi = __builtin_amdgcn_readfirstlane((u32)(x >> 32));
  return ((u64)hi << 32) | lo;
}

// Unaligned little-endian u32 from LDS at byte offset a (>= 0) of an LDS byte array whose base
// is 4-byte aligned: two ds_read_b32 + v_alignbyte.
__device__ __forceinline__ u32 lds_u32(const uint8_t* base, u32 a) {
  const u32* p = reinterpret_cast<const u32*>(base + (a & ~3u));
  return __builtin_amdgcn_alignbyte(p[1], p[0], a & 3u);
}
// Big-endian u16 at byte offset a (bytes::Buf::get_u16).
__device__ __forceinline__ u32 lds_be16(const uint8_t* base, u32 a) {
  u32 w = lds_u32(base, a);
  return ((w & 0xFFu) << 8) | ((w >> 8) & 0xFFu);
}
__device__ __forceinline__ u32 bswap32(u32 w) { return __builtin_bswap32(w); }

// ------------------------------------------------------------------ CRC-32 (table driven)
// tab = kNumCrcTables x 256 u32 in LDS. T_k[b] = R0(b || 0^k): raw CRC (init 0, no xorout).
// ids 0..15: T_0..T_15 (slice-by-16); ids 16+4(j-1)+i (j=1..6): T_{n-1-i}, n = 16<<j.
__device__ __forceinline__ u32 tlook(const u32* tab, int id, u32 byte) { return tab[id * 256 + byte]; }

// R0 of one 16-byte chunk (little-endian dwords w0..w3): XOR_i T_{15-i}[c_i].
__device__ __forceinline__ u32 slice16(const u32* tab, u32 w0, u32 w1, u32 w2, u32 w3) {
  u32 c = tlook(tab, 15, w0 & 0xFF) ^ tlook(tab, 14, (w0 >> 8) & 0xFF) ^
          tlook(tab, 13, (w0 >> 16) & 0xFF) ^ tlook(tab, 12, w0 >> 24);
  c ^= tlook(tab, 11, w1 & 0xFF) ^ tlook(tab, 10, (w1 >> 8) & 0xFF) ^
       tlook(tab, 9, (w1 >> 16) & 0xFF) ^ tlook(tab, 8, w1 >> 24);
  c ^= tlook(tab, 7, w2 & 0xFF) ^ tlook(tab, 6, (w2 >> 8) & 0xFF) ^
       tlook(tab, 5, (w2 >> 16) & 0xFF) ^ tlook(tab, 4, w2 >> 24);
  c ^= tlook(tab, 3, w3 & 0xFF) ^ tlook(tab, 2, (w3 >> 8) & 0xFF) ^
       tlook(tab, 1, (w3 >> 16) & 0xFF) ^ tlook(tab, 0, w3 >> 24);
  return c;
}

// shift_n(A) = R_A(0^n) = XOR_i T_{n-1-i}[byte_i(A)], n = 16 << J.
template <int J>
__device__ __forceinline__ u32 crc_shift(const u32* tab, u32 a) {
  constexpr int b0 = J == 0 ? 15 : 16 + 4 * (J - 1);
  constexpr int d = J == 0 ? -1 : 1;
  return tlook(tab, b0, a & 0xFF) ^ tlook(tab, b0 + d, (a >> 8) & 0xFF) ^
         tlook(tab, b0 + 2 * d, (a >> 16) & 0xFF) ^ tlook(tab, b0 + 3 * d, a >> 24);
}

// 16 bytes starting at signed LDS byte offset x (relative to win); e = x & 15 is wave-uniform.
__device__ __forceinline__ void lds_chunk16(const uint8_t* win, int x, u32 e, u32& o0, u32& o1,
                                            u32& o2, u32& o3) {
  const uint4* p = reinterpret_cast<const uint4*>(win + (x & ~15));
  uint4 a = p[0], b = p[1];
  u32 s = e & 3u, q = e >> 2;
  u32 w0, w1, w2, w3, w4;
  if (q == 0) { w0 = a.x; w1 = a.y; w2 = a.z; w3 = a.w; w4 = b.x; }
  else if (q == 1) { w0 = a.y; w1 = a.z; w2 = a.w; w3 = b.x; w4 = b.y; }
  else if (q == 2) { w0 = a.z; w1 = a.w; w2 = b.x; w3 = b.y; w4 = b.z; }
  else { w0 = a.w; w1 = b.x; w2 = b.y; w3 = b.z; w4 = b.w; }
  o0 = __builtin_amdgcn_alignbyte(w1, w0, s);
  o1 = __builtin_amdgcn_alignbyte(w2, w1, s);
  o2 = __builtin_amdgcn_alignbyte(w3, w2, s);
  o3 = __builtin_amdgcn_alignbyte(w4, w3, s);
}

// keep the bytes of dword at payload position pos (4 bytes) that are >= 0
__device__ __forceinline__ u32 mask_front(u32 w, int pos) {
  if (pos >= 0) return w;
  if (pos <= -4) return 0u;
  return w & (~0u << (8 * (-pos)));
}

// CRC-32 of the payload at LDS offset pb (relative to win), length P >= 4, whose first four
// bytes have already been complemented (init 0xFFFFFFFF folded into the message).
// Returns ~R0(payload') in every lane.
__device__ __forceinline__ u32 wave_crc(const u32* tab, const uint8_t* win, int pb, u32 P) {
  const u32 lane = lane_id();
  const u32 G = (P + 15) >> 4;          // chunks, end-aligned
  const u32 R = (G + 63) >> 6;          // rounds of 64 chunks
  const u32 e = (u32)(pb + (int)P) & 15u;
  u32 A = 0;
  for (u32 r = R; r-- > 0;) {
    const u32 g = lane + 64u * r;
    u32 c = 0;
    if (g < G) {
      const int start = (int)P - 16 * (int)(g + 1);
      u32 w0, w1, w2, w3;
      lds_chunk16(win, pb + start, e, w0, w1, w2, w3);
      w0 = mask_front(w0, start);
      w1 = mask_front(w1, start + 4);
      w2 = mask_front(w2, start + 8);
      w3 = mask_front(w3, start + 12);
      c = slice16(tab, w0, w1, w2, w3);
    }
    A = (r + 1 == R) ? c : (crc_shift<6>(tab, A) ^ c);
  }
  // lane tree: result = XOR_l shift_{16 l}(A_l)
  u32 y;
  y = __shfl_down(A, 1);  if ((lane & 1u) == 0) A ^= crc_shift<0>(tab, y);
  y = __shfl_down(A, 2);  if ((lane & 3u) == 0) A ^= crc_shift<1>(tab, y);
  y = __shfl_down(A, 4);  if ((lane & 7u) == 0) A ^= crc_shift<2>(tab, y);
  y = __shfl_down(A, 8);  if ((lane & 15u) == 0) A ^= crc_shift<3>(tab, y);
  y = __shfl_down(A, 16); if ((lane & 31u) == 0) A ^= crc_shift<4>(tab, y);
  y = __shfl_down(A, 32); if ((lane & 63u) == 0) A ^= crc_shift<5>(tab, y);
  return ~uni(A);
}

// ------------------------------------------------------------------ entry tables
// Wave path: per entry one u32 per column, (end << 16) | src, both < 65536 (block <= 5104 B).
// Big path: per entry one uint2 per column, {end, src}.
struct TabSmall {
  u32* k;
  u32* v;
  __device__ __forceinline__ void put(u32 i, u32 kend, u32 ksrc, u32 vend, u32 vsrc) const {
    k[i] = (kend << 16) | ksrc;
    v[i] = (vend << 16) | vsrc;
  }
  __device__ __forceinline__ u32 end(bool val, u32 j) const { return (val ? v[j] : k[j]) >> 16; }
  __device__ __forceinline__ void get(bool val, u32 j, u32& end, u32& src) const {
    u32 t = val ? v[j] : k[j];
    end = t >> 16;
    src = t & 0xFFFFu;
  }
};
// Big path: per entry one u64 per column, {end, src}, in this workgroup's global scratch.
// Written and read back by the same wave: stores are drained (s_waitcnt vmcnt(0)) before the
// copy phase and reads use sc1 (L2-served) loads, so no stale L1 line of a previous block's
// table can be returned.
struct TabBig {
  u64* k;
  u64* v;
  __device__ __forceinline__ void put(u32 i, u32 kend, u32 ksrc, u32 vend, u32 vsrc) const {
    k[i] = ((u64)ksrc << 32) | kend;
    v[i] = ((u64)vsrc << 32) | vend;
  }
  __device__ __forceinline__ u64 ld(bool val, u32 j) const {
    return __hip_atomic_load(val ? v + j : k + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __device__ __forceinline__ u32 end(bool val, u32 j) const { return (u32)ld(val, j); }
  __device__ __forceinline__ void get(bool val, u32 j, u32& end, u32& src) const {
    u64 t = ld(val, j);
    end = (u32)t;
    src = (u32)(t >> 32);
  }
};

// wave-inclusive prefix sum over 64 lanes
__device__ __forceinline__ u32 wave_scan_incl(u32 x) {
  const u32 lane = lane_id();
#pragma unroll
  for (u32 d = 1; d < 64; d <<= 1) {
    u32 t = __shfl_up(x, d);
    if (lane >= d) x += t;
  }
  return x;
}

// ------------------------------------------------------------------ per-block decode
struct Out {
  uint8_t* keys;
  uint8_t* vals;
  u32* kend;
  u32* vend;
  u32* count;
  uint8_t* status;
  u32* crc;
  u32* defer_list;
  u32* defer_count;
};

__device__ __forceinline__ void put_meta(const Out& o, u32 b, u32 st, u32 n, u32 crc) {
  if (lane_id() == 0) {
    o.status[b] = (uint8_t)st;
    o.count[b] = n;
    o.crc[b] = crc;
  }
}

// Output-driven copy of one column: lane handles 16-byte chunks c = lane, lane+64, ...
// Byte x of the column comes from segment j = first entry with end_j > x, at LDS offset
// src_j + (x - start_j) (relative to win). Empty segments (tombstone values) are skipped by
// the end_j > x search.
template <class Tab>
__device__ __forceinline__ void copy_column(const uint8_t* win, const Tab& tab, bool val, u32 n,
                                            u32 tot, uint8_t* dst) {
  const u32 lane = lane_id();
  const u32 nchunks = (tot + 15) >> 4;
  u32 top = 1;
  while (top * 2 <= n) top *= 2;
  for (u32 c0 = 0; c0 < nchunks; c0 += 64) {
    const u32 c = c0 + lane;
    if (c >= nchunks) break;
    const u32 x0 = c * 16;
    // j = #entries with end <= x0 (upper bound), fixed-step binary search
    u32 j = 0;
    for (u32 step = top; step; step >>= 1)
      if (j + step <= n && tab.end(val, j + step - 1) <= x0) j += step;
    u32 end, src, st;
    tab.get(val, j, end, src);
    st = j ? tab.end(val, j - 1) : 0;
    u32 w[4];
#pragma unroll
    for (int d = 0; d < 4; d++) {
      const u32 x = x0 + 4 * d;
      u32 word = 0;
      if (x < tot) {
        while (end <= x && j + 1 < n) { st = end; j++; tab.get(val, j, end, src); }
        if (x + 4 <= end) {
          word = lds_u32(win, src + (x - st));
        } else {
#pragma unroll
          for (u32 bb = 0; bb < 4; bb++) {
            const u32 xb = x + bb;
            if (xb < tot) {
              while (end <= xb && j + 1 < n) { st = end; j++; tab.get(val, j, end, src); }
              word |= (u32)win[src + (xb - st)] << (8 * bb);
            }
          }
        }
      }
      w[d] = word;
    }
    *reinterpret_cast<uint4*>(dst + x0) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// Decode the block whose bytes are at win[a0 .. a0+len) (LDS), block index b.
// Returns true when the block was handed to the big path instead.
template <class Tab, bool BIG>
__device__ __forceinline__ bool decode_block(const u32* tab, uint8_t* win, const Tab& et, u32 a0,
                                             u32 len, u32 b, u64 ext_b, const Out& o) {
  const u32 lane = lane_id();
  if (len == 0) { put_meta(o, b, TPZ_BLOCK_EMPTY, 0, 0); return false; }           // compress.rs:96
  const u32 tag = win[a0 + len - 1];                                                 // compress.rs:99
  if (tag == 0 || tag > 3) { put_meta(o, b, TPZ_BLOCK_BAD_TAG, 0, 0); return false; } // :44-53,102
  if (tag != 1) { put_meta(o, b, TPZ_BLOCK_UNSUPPORTED_CODEC, 0, 0); return false; }
  if (len - 1 < 4) { put_meta(o, b, TPZ_BLOCK_MALFORMED, 0, 0); return false; }     // block.rs:49
  const u32 P = len - 5;
  const int pb = (int)a0;
  const u32 stored = bswap32(lds_u32(win, a0 + P));                                  // block.rs:51
  u32 crc;
  if (P >= 4) {
    // fold init 0xFFFFFFFF into the first four payload bytes, compute, restore
    if (lane < 4) win[a0 + lane] ^= 0xFFu;
    __builtin_amdgcn_wave_barrier();
    crc = wave_crc(tab, win, pb, P);
    __builtin_amdgcn_wave_barrier();
    if (lane < 4) win[a0 + lane] ^= 0xFFu;
    __builtin_amdgcn_wave_barrier();
  } else {
    u32 c = 0xFFFFFFFFu;
    for (u32 i = 0; i < P; i++) {
      c ^= win[a0 + i];
      for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    }
    crc = ~c;
  }
  if (crc != stored) { put_meta(o, b, TPZ_BLOCK_CHECKSUM_MISMATCH, 0, crc); return false; }
  if (P < 2) { put_meta(o, b, TPZ_BLOCK_MALFORMED, 0, crc); return false; }          // block.rs:54
  const u32 n = lds_be16(win, a0);
  if (P < 2 + 2 * n) { put_meta(o, b, TPZ_BLOCK_MALFORMED, 0, crc); return false; }  // :56-59
  if (!BIG && n > kWaveMaxN) {
    if (lane == 0) o.defer_list[atomicAdd(o.defer_count, 1u)] = b;
    return true;
  }
  const u32 db = a0 + 2 + 2 * n;   // entries region (Block.data), LDS offset
  const u32 dl = P - 2 - 2 * n;
  const bool slots_fit = 6u * n <= len;
  u32* kend_g = o.kend + slot_base(ext_b, b);
  u32* vend_g = o.vend + slot_base(ext_b, b);
  u32 kc = 0, vc = 0;
  bool bad = false;
  for (u32 g0 = 0; g0 < n; g0 += 64) {
    const u32 i = g0 + lane;
    const bool act = i < n;
    u32 off = 0, kl = 0, vl = 0;
    bool ok = true;
    if (act) {
      off = lds_be16(win, a0 + 2 + 2 * i);                                          // iterator.rs:74
      ok = off + 2 <= dl;
      if (ok) { kl = lds_be16(win, db + off); ok = off + 4 + kl <= dl; }            // :77-81
      if (ok) { vl = lds_be16(win, db + off + 2 + kl); ok = off + 4 + kl + vl <= dl; } // :81-82
      if (!ok) kl = vl = 0;
    }
    bad |= __ballot(act && !ok) != 0;
    const u32 ki = wave_scan_incl(kl) + kc;
    const u32 vi = wave_scan_incl(vl) + vc;
    if (act && slots_fit) {
      et.put(i, ki, db + off + 2, vi, db + off + 4 + kl);
      kend_g[i] = ki;
      vend_g[i] = vi;
    }
    kc = __shfl(ki, 63);
    vc = __shfl(vi, 63);
  }
  if (bad) { put_meta(o, b, TPZ_BLOCK_MALFORMED, 0, crc); return false; }
  if (!slots_fit || kc > len || vc > len) { put_meta(o, b, TPZ_BLOCK_OVERLAP, n, crc); return false; }
  if (BIG) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  }
  __builtin_amdgcn_wave_barrier();
  const u64 kb = key_base(ext_b, b);
  copy_column(win, et, false, n, kc, o.keys + kb);
  copy_column(win, et, true, n, vc, o.vals + kb);
  put_meta(o, b, TPZ_BLOCK_OK, n, crc);
  return false;
}

__device__ __forceinline__ void load_tables(u32* tab, const u32* gtab) {
  const uint4* s = reinterpret_cast<const uint4*>(gtab);
  uint4* d = reinterpret_cast<uint4*>(tab);
  for (int i = threadIdx.x; i < kTableBytes / 16; i += blockDim.x) d[i] = s[i];
  __syncthreads();
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t window_rsrc(const uint8_t* src, u64 src_bytes,
                                                               u64 wstart) {
  u64 rem = src_bytes > wstart ? src_bytes - wstart : 0;
  if (rem > 0x7FFFFFF0ull) rem = 0x7FFFFFF0ull;
  return __builtin_amdgcn_make_buffer_rsrc((void*)(src + wstart), (short)0, (int)rem, 0x00020000);
}

// A 16-byte piece that straddles the end of the source buffer comes back zeroed from the
// range-checked buffer load; refill the in-range bytes one by one (only the batch's tail).
__device__ __forceinline__ void fix_tail(uint4& v, const uint8_t* src, u64 piece, u64 src_bytes) {
  if (piece + 16 > src_bytes && piece < src_bytes) {
    u32 w[4] = {0, 0, 0, 0};
    for (u32 k = 0; k < 16 && piece + k < src_bytes; k++) w[k >> 2] |= (u32)src[piece + k] << (8 * (k & 3));
    v = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

struct Params {
  u64* big_scratch;  // gridDim(big) x 2 x kBigMaxSlots u64
  const uint8_t* src;
  const u64* ext;
  u64 src_bytes;
  u32 n_blocks;
  const u32* crc_tables;
  Out out;
};

// ------------------------------------------------------------------ wave path kernel
__global__ __launch_bounds__(kWGThreads, 4) void decode_wave_kernel(Params p) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kWaveLds];
  u32* tab = reinterpret_cast<u32*>(lds);
  load_tables(tab, p.crc_tables);

  const u32 wid = uni(threadIdx.x >> 6);
  const u32 lane = lane_id();
  uint8_t* slot = lds + kTableBytes + wid * kSlotBytes;
  uint8_t* win = slot + kGuard;
  TabSmall et{reinterpret_cast<u32*>(win + kWinBytes + 32),
              reinterpret_cast<u32*>(win + kWinBytes + 32 + kWaveMaxN * 4)};

  const u32 nw = gridDim.x * kWavesPerWG;
  u32 b = blockIdx.x * kWavesPerWG + wid;

  // prefetch state for block b
  uint4 v[kWinRounds];
  u64 s_cur = 0, e_cur = 0;
  auto issue = [&](u32 bb, u64& s, u64& e) {
    if (bb >= p.n_blocks) return;
    s = uni64(p.ext[bb]);
    e = uni64(p.ext[bb + 1]);
    const u64 len = e - s;
    if (len > kWaveMaxLen) return;
    const u64 ws = s & ~15ull;
    const u32 nbytes = (u32)(e - ws);
    const u32 rounds = (nbytes + 1023) >> 10;
    __amdgpu_buffer_rsrc_t rs = window_rsrc(p.src, p.src_bytes, ws);
#pragma unroll
    for (int r = 0; r < kWinRounds; r++)
      if ((u32)r < rounds) v[r] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (u32)(r * 1024 + lane * 16), 0, 0));
    if (e + 16 > p.src_bytes) {
#pragma unroll
      for (int r = 0; r < kWinRounds; r++)
        if ((u32)r < rounds) fix_tail(v[r], p.src, ws + r * 1024 + lane * 16, p.src_bytes);
    }
  };
  issue(b, s_cur, e_cur);

  while (b < p.n_blocks) {
    const u64 s = s_cur, e = e_cur;
    const u32 len64 = (e - s) > 0xFFFFFFFFull ? 0xFFFFFFFFu : (u32)(e - s);
    const bool fits = (e - s) <= kWaveMaxLen;
    if (fits) {
      const u32 rounds = (u32)((e - (s & ~15ull)) + 1023) >> 10;
#pragma unroll
      for (int r = 0; r < kWinRounds; r++)
        if ((u32)r < rounds) *reinterpret_cast<uint4*>(win + r * 1024 + lane * 16) = v[r];
    }
    const u32 bcur = b;
    b += nw;
    issue(b, s_cur, e_cur);          // next block's loads fly while this one decodes
    __builtin_amdgcn_wave_barrier();
    if (fits) {
      decode_block<TabSmall, false>(tab, win, et, (u32)(s & 15u), len64, bcur, s, p.out);
    } else if (len64 > kBigMaxLen) {
      put_meta(p.out, bcur, TPZ_BLOCK_TOO_LARGE, 0, 0);
    } else if (lane == 0) {
      p.out.defer_list[atomicAdd(p.out.defer_count, 1u)] = bcur;
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// ------------------------------------------------------------------ big path kernel
__global__ __launch_bounds__(kWave, 1) void decode_big_kernel(Params p) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kBigLds];
  u32* tab = reinterpret_cast<u32*>(lds);
  load_tables(tab, p.crc_tables);
  const u32 lane = lane_id();
  uint8_t* win = lds + kTableBytes + kGuard;
  TabBig et{p.big_scratch + (u64)blockIdx.x * 2 * kBigMaxSlots,
            p.big_scratch + (u64)blockIdx.x * 2 * kBigMaxSlots + kBigMaxSlots};
  const u32 cnt = uni(*p.out.defer_count);
  for (u32 it = blockIdx.x; it < cnt; it += gridDim.x) {
    const u32 b = uni(p.out.defer_list[it]);
    const u64 s = uni64(p.ext[b]), e = uni64(p.ext[b + 1]);
    const u32 len = (u32)(e - s);
    const u64 ws = s & ~15ull;
    const u32 nbytes = (u32)(e - ws);
    __amdgpu_buffer_rsrc_t rs = window_rsrc(p.src, p.src_bytes, ws);
    for (u32 off = 0; off < nbytes; off += 4096) {
      uint4 t[4];
#pragma unroll
      for (int r = 0; r < 4; r++)
        t[r] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + r * 1024 + lane * 16, 0, 0));
#pragma unroll
      for (int r = 0; r < 4; r++) {
        fix_tail(t[r], p.src, ws + off + r * 1024 + lane * 16, p.src_bytes);
        if (off + r * 1024 < nbytes) *reinterpret_cast<uint4*>(win + off + r * 1024 + lane * 16) = t[r];
      }
    }
    __builtin_amdgcn_wave_barrier();
    decode_block<TabBig, true>(tab, win, et, (u32)(s & 15u), len, b, s, p.out);
    __builtin_amdgcn_wave_barrier();
  }
}

void launch_decode(const LaunchArgs& a, hipStream_t stream) {
  Params p;
  p.src = a.src;
  p.ext = a.ext;
  p.src_bytes = a.src_bytes;
  p.n_blocks = a.n_blocks;
  p.crc_tables = a.crc_tables;
  p.big_scratch = a.big_scratch;
  p.out = Out{a.keys, a.vals, a.kend, a.vend, a.count, a.status, a.crc, a.defer_list, a.defer_count};
  u32 wgs_needed = (a.n_blocks + kWavesPerWG - 1) / kWavesPerWG;
  u32 grid = a.num_cus;
  if (wgs_needed < grid) grid = wgs_needed ? wgs_needed : 1;
  hipLaunchKernelGGL(decode_wave_kernel, dim3(grid), dim3(kWGThreads), 0, stream, p);
  hipLaunchKernelGGL(decode_big_kernel, dim3(a.big_grid), dim3(kWave), 0, stream, p);
}

}  // namespace tpz
