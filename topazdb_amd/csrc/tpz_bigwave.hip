// tpz_bigwave.hip — gfx950 kernel for long blocks with few entries (the 64 KiB config:
// block_size 65536, 61 entries of 32-B keys and 1 KiB values), one wavefront per block.
//
// The LDS big path (tpz_decode.hip, the tail kernel's big phase) stages a whole block in a 92 KiB
// window, so a CU holds one block at a time and its CRC, parse and copy run back to back with the
// next block's bytes only in flight: 0.31 of the HBM roofline on the 64k config, 0.35 for its
// memory skeleton alone. Here nothing is staged. Each wave of a 16-wave workgroup decodes its own
// block straight from HBM, so a CU keeps 16 blocks in flight:
//   * parse (Block::decode, src/block.rs:46-65, and BlockIterator::seek_to's bounds checks,
//     src/block/iterator.rs:74-82): lane i reads offset i, then key and value lengths, from
//     global memory; DPP-free shuffles scan them into the {kend, vend} ends and a per-wave entry
//     table in LDS (<= 128 segments: the wave path routes here only blocks with n <= 63);
//   * copy: the output stream in 1 KiB windows (lane = one 16-byte chunk); a 64-slot chunk map
//     per window, filled by the segments that end in it, gives each chunk its segment by a prefix
//     max (the wave path's scheme, windowed); the chunk's bytes are unaligned 16-byte loads from
//     the block in global memory (coalesced within a segment), merged where segments meet;
//   * CRC (src/checksum.rs:6-21): 8 KiB windows aligned to the payload's padded end; lane l folds
//     the 128-byte run ending 128 l bytes before the window end straight from registers with
//     slice-by-4 lookups into tables replicated 32 times in LDS (lane l reads replica l % 32:
//     bank-conflict-free), shifts it there with one GF(2) multiply by x^(8*128*l) mod P, and the
//     wave XORs the lanes; windows are chained with x^(8*8192). The init value is folded into the
//     first four payload bytes and the bytes past the payload are zeroed in registers, and the
//     result is compared in the shifted domain, as the wave path does.
// Blocks whose entries overlap or overrun the slot go to the spill path, as everywhere else.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tpz_internal.h"

// copy/CRC pipeline shape (variants: tools/abl_multi.py)
// (measured on the 64k config, profiles/r2/bw_shapes.log: 16 waves, one group at a time, 4 KiB
// copy groups and 4 KiB CRC steps 2.16 ms; 12 waves with 6 KiB 2.21; 8 waves with 8 KiB 2.32;
// two 2 KiB groups in flight 2.50; two 4 KiB groups spill VGPRs)
#ifndef TPZ_BW_KU
#define TPZ_BW_KU 4
#endif
#ifndef TPZ_BW_STEPRUN
#define TPZ_BW_STEPRUN 64
#endif
#ifndef TPZ_BW_PIPE
#define TPZ_BW_PIPE 0
#endif

namespace tpz {

namespace bw {

typedef uint32_t u32;
typedef uint64_t u64;

constexpr int kWave = 64;
#ifndef TPZ_BW_WAVES
#define TPZ_BW_WAVES 16
#endif
constexpr int kWaves = TPZ_BW_WAVES;              // waves per workgroup (one workgroup per CU)
constexpr int kThreads = kWave * kWaves;
constexpr u32 kRun = 128;                         // CRC bytes per lane per window (256: VGPR spills)
constexpr u32 kCrcWin = kRun * kWave;             // 8 KiB
constexpr u32 kStepRun = TPZ_BW_STEPRUN;          // fused CRC: bytes per lane per step
constexpr int kStepPieces = kStepRun / 16;
constexpr u32 kStep = kStepRun * kWave;           // 4 KiB per step, one step per copy group
constexpr int kSegs = 128;                        // entry-table slots per wave (2 n <= 126, + 2 sentinels)
constexpr int kU = TPZ_BW_KU;                     // copy windows per group
constexpr int kWaveLds = kSegs * 8 + kU * kWave;   // entry table + kU u8 chunk maps
constexpr int kShiftWords = 4 * 256;                // the step shift's byte tables (x^(8 kStep))
constexpr int kLdsBytes = kCrcRepWords * 4 + kWaves * kWaveLds + kShiftWords * 4;
static_assert(kLdsBytes <= 163840, "bigwave LDS");
constexpr u32 kOob = 0x80000000u;

// The lane id, laundered: masks and offsets derived from it are recomputed where they are used
// instead of being hoisted out of the block loop into SGPR pairs that spill (tpz_decode.hip).
__device__ __forceinline__ u32 lane_id() {
  u32 l = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  asm volatile("" : "+v"(l));
  return l;
}
__device__ __forceinline__ u32 uni(u32 x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ u32 readlane(u32 x, u32 l) { return __builtin_amdgcn_readlane(x, l); }
__device__ __forceinline__ u32 xor3(u32 a, u32 b, u32 c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// a * b mod P, reflected (bit 31 = x^0), per lane (the multiplier varies across lanes).
__device__ __forceinline__ u32 gf_mul(u32 a, u32 b) {
  u32 p = 0;
#pragma unroll
  for (int i = 0; i < 32; i++) {
    const u32 m = (u32)((int)(a << i) >> 31);
    p ^= b & m;
    b = (b >> 1) ^ (0xEDB88320u & (u32)(-(int)(b & 1u)));
  }
  return p;
}

__device__ __forceinline__ u32 wave_xor(u32 x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x ^= __shfl_xor(x, o, kWave);
  return x;
}
// wave scans with DPP row shifts and row broadcasts (lanes past a row's start read 0)
template <int CTRL>
__device__ __forceinline__ u32 dpp(u32 x) {
  return (u32)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, true);
}
constexpr int kRowShr = 0x110, kRowBcast15 = 0x142, kRowBcast31 = 0x143;
__device__ __forceinline__ u32 scan_incl(u32 x) {
  x += dpp<kRowShr + 1>(x);
  x += dpp<kRowShr + 2>(x);
  x += dpp<kRowShr + 4>(x);
  x += dpp<kRowShr + 8>(x);
  x += (u32)__builtin_amdgcn_update_dpp(0, (int)x, kRowBcast15, 0xA, 0xF, false);
  x += (u32)__builtin_amdgcn_update_dpp(0, (int)x, kRowBcast31, 0xC, 0xF, false);
  return x;
}
__device__ __forceinline__ u32 scan_max(u32 x) {
  x = max(x, dpp<kRowShr + 1>(x));
  x = max(x, dpp<kRowShr + 2>(x));
  x = max(x, dpp<kRowShr + 4>(x));
  x = max(x, dpp<kRowShr + 8>(x));
  x = max(x, (u32)__builtin_amdgcn_update_dpp(0, (int)x, kRowBcast15, 0xA, 0xF, false));
  x = max(x, (u32)__builtin_amdgcn_update_dpp(0, (int)x, kRowBcast31, 0xC, 0xF, false));
  return x;
}
// LDS written by this wave and read back by other lanes of it: the LDS executes one wave's
// instructions in order, so only the compiler must keep them in order. (A wavefront-scope fence
// makes the compiler wait for every outstanding global load and store, s_waitcnt vmcnt(0), which
// drained the copy pipeline at every window group: 3.0 ms vs ... on the 64k config.)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ u32 lanes_below(u64 mask) {
  return __builtin_amdgcn_mbcnt_hi((u32)(mask >> 32), __builtin_amdgcn_mbcnt_lo((u32)mask, 0u));
}

// One slice-by-4 step (tpz_crc.hip's layout: word ((t*256 + b)*32 + r) = T_t[b]).
__device__ __forceinline__ u32 slice4(const u32* rep, u32 r, u32 x) {
  const u32 a0 = rep[((3u * 256u + (x & 0xFF)) << 5) + r];
  const u32 a1 = rep[((2u * 256u + ((x >> 8) & 0xFF)) << 5) + r];
  const u32 a2 = rep[((1u * 256u + ((x >> 16) & 0xFF)) << 5) + r];
  const u32 a3 = rep[((x >> 24) << 5) + r];
  return xor3(a0, a1, a2) ^ a3;
}

// bytes [lo, hi) of a 16-byte piece (clamped to 0..16) as a mask pair
__device__ __forceinline__ void range_mask(int lo, int hi, u64& mlo, u64& mhi) {
  lo = lo < 0 ? 0 : (lo > 16 ? 16 : lo);
  hi = hi < 0 ? 0 : (hi > 16 ? 16 : hi);
  auto upto = [](int k) -> u64 { return k >= 8 ? ~0ull : ((1ull << (8 * k)) - 1); };
  const u64 below_hi_lo = upto(hi), below_lo_lo = upto(lo);
  const u64 below_hi_hi = hi <= 8 ? 0ull : upto(hi - 8), below_lo_hi = lo <= 8 ? 0ull : upto(lo - 8);
  mlo = below_hi_lo & ~below_lo_lo;
  mhi = below_hi_hi & ~below_lo_hi;
}

#ifdef TPZ_BW_STAMPS
// diagnostic build: per-phase wave cycles summed over the grid (parse, map, loads issue, merge +
// store, CRC, other)
__device__ unsigned long long g_bw_stamps[8];
#define BW_T0() u64 tq_ = __builtin_amdgcn_s_memtime()
#define BW_ST(i) do { const u64 n_ = __builtin_amdgcn_s_memtime(); st_[i] += n_ - tq_; tq_ = n_; } while (0)
#else
#define BW_T0() (void)0
#define BW_ST(i) (void)0
#endif

struct BWParams {
  const uint8_t* src;
  const u64* ext;
  u64 src_bytes;
  const u32* rep;           // replicated slice-by-4 tables (kCrcRepWords)
  const u32* tab;           // the decode tables (T_0..T_3 and the inverse table, global)
  const u32* list;
  uint8_t* data;
  u32* ends;
  u32* count;
  uint8_t* status;
  u32* crc;
  u32* spill_list;
  u32* spill_count;
  u32* big_list;
  u32* big_count;
  const u64* efirst;        // exact ends layout, or null: slotted
  u32 lane_shift[64];       // x^(8 * 128 l) mod P
  u32 win_shift;            // x^(8 * 8192) mod P
  u32 half_shift;           // x^(8 * 64) mod P
  u32 step_lane_shift[64];  // x^(8 * 64 l) mod P (the fused CRC steps' lane runs)
  u32 step_shift;           // x^(8 * 4096) mod P
};

__device__ __forceinline__ u32 gtab(const BWParams& p, int id, u32 b) { return p.tab[id * 256 + b]; }
__device__ __forceinline__ u32 shift_small(const BWParams& p, u32 a, u32 k) {
  u32 r = k >= 4 ? 0u : (a >> (8 * k));
  for (u32 i = 0; i < 4 && i < k; i++) r ^= gtab(p, (int)(k - 1 - i), (a >> (8 * i)) & 0xFF);
  return r;
}
__device__ __forceinline__ u32 unshift_small(const BWParams& p, u32 r, u32 k) {
  for (u32 i = 0; i < k; i++) {
    const u32 b = gtab(p, kCrcInvTable, r >> 24);
    r = ((r ^ gtab(p, 0, b)) << 8) | b;
  }
  return r;
}

__device__ __forceinline__ u32 be16_at(const uint8_t* q) { return ((u32)q[0] << 8) | q[1]; }

// A block's header words: lane l < 33 holds block bytes [4 l, 4 l + 4) (n and up to 63 offsets),
// lane 62 the four bytes of the stored CRC, lane 63 the last four bytes (the tag on top).
// Wave-uniform reads of memory no kernel of the decode writes while the tail kernel runs (the
// extents; the bigwave list, complete before it starts): through the constant address space, so
// they are scalar loads even though the kernel also issues atomics and stores (the compiler
// otherwise makes them vector loads, whose waits drained the copy pipeline: 64k 2.31 vs 2.11 ms).
template <class T>
__device__ __forceinline__ T ld_uniform(const T* base, u64 i) {
  return reinterpret_cast<const __attribute__((address_space(4))) T*>(reinterpret_cast<uintptr_t>(base))[i];
}

__device__ __forceinline__ u32 hdr_load(const BWParams& p, u64 s, u64 e) {
  const u32 lane = lane_id(), len = (u32)(e - s);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.src + s), (short)0, (int)len, 0x00020000);
  const u32 off = lane < 33 ? 4 * lane : (lane == 62 ? len - 5 : (lane == 63 ? len - 4 : kOob));
  return (u32)__builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
}

__device__ __forceinline__ void put_meta(const BWParams& p, u32 b, u32 st, u32 n, u32 crc) {
  if (lane_id() == 0) {
    p.status[b] = (uint8_t)st;
    p.count[b] = n;
    p.crc[b] = crc;
  }
}

// R0(payload' || 0^k) of the block's payload [s, s + P), payload' = the payload with its first
// four bytes complemented, padded with k zero bytes to the next 16-byte boundary of the address.
__device__ __forceinline__ u32 block_crc(const BWParams& p, const u32* rep, u64 s, u32 P) {
  const u32 lane = lane_id();
  const u64 pend = s + P, Pa = (pend + 15) & ~15ull;      // padded end, 16-aligned
  const u64 base = s & ~15ull;
  const u64 lim = (p.src_bytes < Pa ? p.src_bytes : Pa) - base;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.src + base), (short)0, (int)(lim < 0x7FFFFFF0ull ? lim : 0x7FFFFFF0ull), 0x00020000);
  const u32 W = (u32)((Pa - base + kCrcWin - 1) / kCrcWin);
  const u32 ls = p.lane_shift[lane];
  u32 acc = 0;
  for (u32 wi = W; wi-- > 0;) {                            // lowest window first
    const u64 wend = Pa - (u64)kCrcWin * wi;
    const u64 r0 = wend - (u64)kRun * (lane + 1);         // this lane's run [r0, r0 + kRun)
    uint4 v[kRun / 16];
#pragma unroll
    for (int t = 0; t < (int)(kRun / 16); t++) {
      const u64 a = r0 + 16 * t;
      v[t] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                           rs, (int64_t)a >= (int64_t)base ? (u32)(a - base) : kOob, 0, 0));
    }
    // keep payload bytes [s, pend) only; complement bytes [s, s + 4) (the init value): only the
    // highest window and the windows that start before s + 4 (the lowest, and the next one when
    // [s, s + 4) crosses into it) hold such pieces
    if (wi == 0 || (int64_t)(wend - kCrcWin) < (int64_t)(s + 4)) {
#pragma unroll
    for (int t = 0; t < (int)(kRun / 16); t++) {
      const u64 a = r0 + 16 * t;
      if (a < s + 4 || a + 16 > pend) {
        u64 klo, khi, xlo, xhi;
        range_mask((int)((int64_t)s - (int64_t)a), (int)((int64_t)pend - (int64_t)a), klo, khi);
        range_mask((int)((int64_t)s - (int64_t)a), (int)((int64_t)s + 4 - (int64_t)a), xlo, xhi);
        u64 lo = (u64)v[t].y << 32 | v[t].x, hi = (u64)v[t].w << 32 | v[t].z;
        lo = (lo & klo) ^ xlo;
        hi = (hi & khi) ^ xhi;
        v[t] = make_uint4((u32)lo, (u32)(lo >> 32), (u32)hi, (u32)(hi >> 32));
      }
    }
    }
    // two independent chains (the run's halves) halve the lookup latency chain; the first half
    // is shifted past the second with x^(8*64)
    u32 ca = 0, cb = 0;
    const u32 r = lane & 31;
    constexpr int H = kRun / 32;
#pragma unroll
    for (int t = 0; t < H; t++) {
      ca = slice4(rep, r, ca ^ v[t].x);
      cb = slice4(rep, r, cb ^ v[t + H].x);
      ca = slice4(rep, r, ca ^ v[t].y);
      cb = slice4(rep, r, cb ^ v[t + H].y);
      ca = slice4(rep, r, ca ^ v[t].z);
      cb = slice4(rep, r, cb ^ v[t + H].z);
      ca = slice4(rep, r, ca ^ v[t].w);
      cb = slice4(rep, r, cb ^ v[t + H].w);
    }
    const u32 c = gf_mul(p.half_shift, ca) ^ cb;
    const u32 part = wave_xor(gf_mul(ls, c));
    acc = (wi + 1 == W) ? part : (gf_mul(p.win_shift, acc) ^ part);
  }
  return acc;
}

// The 16 bytes at descriptor offset c (the block starts at sa in the descriptor, 16..31 bytes in
// unless the block starts within 16 bytes of d_src). A chunk's second piece is its segment's source
// shifted back by up to 15 bytes, so c < 0 only for a block at the very start of d_src; those
// leading bytes read as zero (they are masked out by the merge anyway).
__device__ __forceinline__ uint4 seg_load(__amdgpu_buffer_rsrc_t rs, int c, bool on) {
#ifdef TPZ_BW_NOLOAD
  return make_uint4(c, c, on, 7);                     // timing build only
#endif
  const uint4 v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                rs, on ? (u32)(c < 0 ? 0 : c) : kOob, 0, 0));
  if (c >= 0) return v;
  const u32 sh = (u32)(-c) * 8;                       // 8..120 bits
  u64 lo = (u64)v.y << 32 | v.x, hi = (u64)v.w << 32 | v.z;
  if (sh >= 64) {
    hi = lo << (sh - 64);
    lo = 0;
  } else {
    hi = (hi << sh) | (lo >> (64 - sh));
    lo <<= sh;
  }
  return make_uint4((u32)lo, (u32)(lo >> 32), (u32)hi, (u32)(hi >> 32));
}

// bytes [0, k) of a, bytes [k, 16) of b (k in 0..16)
__device__ __forceinline__ u32 keep_mask(u32 k, u32 d) {
  const int sel = (int)k - 4 * (int)d;
  return sel >= 4 ? 0xFFFFFFFFu : (sel <= 0 ? 0u : ~(0xFFFFFFFFu << (8 * sel)));
}
__device__ __forceinline__ uint4 merge16(uint4 a, uint4 b, u32 k) {
  return make_uint4((a.x & keep_mask(k, 0)) | (b.x & ~keep_mask(k, 0)),
                    (a.y & keep_mask(k, 1)) | (b.y & ~keep_mask(k, 1)),
                    (a.z & keep_mask(k, 2)) | (b.z & ~keep_mask(k, 2)),
                    (a.w & keep_mask(k, 3)) | (b.w & ~keep_mask(k, 3)));
}

struct Seg {
  u32 end;      // exclusive end in the output stream (0xFFFFFFFF: the sentinels past the last)
  int delta;    // (offset of its first byte in the descriptor) - (its start in the stream)
};

// One group of kU 1 KiB output windows, mapped and loaded (its merges and stores come later, so
// the next group's loads are in flight while this group's stores drain).
struct Group {
  uint4 a[kU], b[kU];
  u32 kj[kU];   // bytes of the chunk from a (16: all of it) | the segment after the chunk's
                // first one << 8 (for chunks that meet 3+ segments)
  bool more;    // some chunk meets 3+ segments (segments under 16 B)
};

// Maps windows w0 .. w0 + kU - 1 to segments and issues their loads. m0 = the number of segments
// ending at or before the group's first chunk start minus 16 (every segment from m0 on ends in or
// after the group's first chunk slot). Segment k ending at stream byte E marks chunk slot
// ceil(E / 16) (relative to the group) with k + 1 (an LDS max: two segments ending in one chunk
// leave the later); a prefix max per window, carried across windows, is then the number of
// segments ending at or before each chunk's start: the index of the segment holding its first
// byte. Returns m0 for the next group.
__device__ __forceinline__ u32 map_group(u32 w0, u32 m0, u32 nseg, const Seg* seg, uint8_t* cmap,
                                         __amdgpu_buffer_rsrc_t rs, Group& g) {
  const u32 lane = lane_id();
#pragma unroll
  for (int i = 0; i < kU * kWave / 16; i += kWave)
    if (i + (int)lane < kU * kWave / 16) reinterpret_cast<uint4*>(cmap)[i + lane] = make_uint4(0, 0, 0, 0);
  wave_lds_sync();
  for (u32 k0 = m0;; k0 += kWave) {
    const u32 k = k0 + lane;
    const u32 E = seg[k < nseg ? k : nseg].end;
    const u32 rel = k < nseg ? ((E + 15) >> 4) - 64 * w0 : 0xFFFFFFFFu;
    // segments end in increasing order: of those ending in one slot only the last writes
    const u32 En = seg[k + 1 < nseg ? k + 1 : nseg].end;
    const u32 reln = k + 1 < nseg ? ((En + 15) >> 4) - 64 * w0 : 0xFFFFFFFFu;
    if (rel < 64u * kU && rel != reln) cmap[rel] = (uint8_t)(k + 1);
    if (k0 + kWave >= nseg || readlane(rel, 63) >= 64u * kU) break;   // wave-uniform
  }
  wave_lds_sync();
  u32 carry = m0;
  bool more = false;
#pragma unroll
  for (int u = 0; u < kU; u++) {
    const u32 x0 = 1024 * (w0 + u) + 16 * lane;
    const u32 j = max(scan_max(cmap[u * kWave + lane]), carry);     // <= nseg (< 128)
    carry = readlane(j, 63);
    const Seg g0 = seg[j], g1 = seg[j + 1];                         // sentinels past nseg
    const bool two = g0.end < x0 + 16;
    more |= two && g1.end < x0 + 16;
    g.kj[u] = (two ? g0.end - x0 : 16u) | ((j + 1) << 8);
    g.a[u] = seg_load(rs, (int)x0 + g0.delta, j < nseg);
    g.b[u] = seg_load(rs, (int)x0 + g1.delta, two);
  }
  g.more = __ballot(more) != 0;
  return carry;
}

// Merges and stores a mapped group: 64 lanes x 16 B per window, through a descriptor that ends at
// the slot's last 128-byte line (chunks past it are dropped; bytes past the stream are zero).
__device__ __forceinline__ void store_group(u32 w0, u32 tot, u32 nseg, const Seg* seg,
                                            __amdgpu_buffer_rsrc_t rs,
                                            __amdgpu_buffer_rsrc_t ds, const Group& g) {
  const u32 lane = lane_id();
#pragma unroll
  for (int u = 0; u < kU; u++) {
    const u32 x0 = 1024 * (w0 + u) + 16 * lane;
    const u32 kk = g.kj[u] & 0xFFu;
    uint4 v = merge16(g.a[u], g.b[u], kk);
    if (g.more) {
      // chunks meeting 3+ segments (segments under 16 B): the rest one by one
      u32 jj = g.kj[u] >> 8;
      u32 e = seg[jj].end;
      if (kk < 16u) {
        while (e < x0 + 16 && jj + 1 < nseg) {
          jj++;
          const Seg s = seg[jj];
          v = merge16(v, seg_load(rs, (int)x0 + s.delta, true), e - x0);
          e = s.end;
        }
      }
    }
    if (1024 * (w0 + u + 1) > tot)                                  // the stream's end
      v = merge16(v, make_uint4(0, 0, 0, 0), x0 < tot ? min(tot - x0, 16u) : 0u);
#ifdef TPZ_BW_NOSTORE
    if (v.x == 0x9E3779B9u && v.y == 0x12345u)
#endif
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) u32, v),
                                           ds, x0, 0, 0);
  }
}

// The CRC fused into the copy loop: 4 KiB steps aligned to the payload's padded end Pa, lowest
// first, one per copy group, so a step reads the source bytes the copy has just read (from L2 or
// the Infinity Cache instead of HBM). Lane l folds the 64-byte run ending 64 l bytes before the
// step's end; its raw CRCs are chained across steps per lane (Horner with x^(8*4096)), and the
// lanes are shifted to Pa and XORed once per block.
struct FusedCrc {
  __amdgpu_buffer_rsrc_t rs;   // [base, min(src_bytes, Pa))
  u64 s, pend, Pa, base;
  u32 S;                       // steps
};

__device__ __forceinline__ FusedCrc fused_crc_init(const BWParams& p, u64 s, u32 P) {
  FusedCrc c;
  c.s = s;
  c.pend = s + P;
  c.Pa = (c.pend + 15) & ~15ull;
  c.base = s & ~15ull;
  const u64 lim = (p.src_bytes < c.Pa ? p.src_bytes : c.Pa) - c.base;
  c.rs = __builtin_amdgcn_make_buffer_rsrc((void*)(p.src + c.base), (short)0,
                                           (int)(lim < 0x7FFFFFF0ull ? lim : 0x7FFFFFF0ull), 0x00020000);
  c.S = (u32)((c.Pa - c.base + kStep - 1) / kStep);
  return c;
}

__device__ __forceinline__ void fused_crc_issue(const FusedCrc& c, u32 i, uint4 (&v)[kStepPieces]) {
  const u64 wend = c.Pa - (u64)kStep * (c.S - 1 - i);
  const u64 r0 = wend - (u64)kStepRun * (lane_id() + 1);
#pragma unroll
  for (int t = 0; t < kStepPieces; t++) {
    const u64 a = r0 + 16 * t;
    v[t] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                         c.rs, (int64_t)a >= (int64_t)c.base ? (u32)(a - c.base) : kOob, 0, 0));
  }
}

__device__ __forceinline__ u32 fused_crc_fold(const FusedCrc& c, const BWParams& p, const u32* rep,
                                              u32 i, uint4 (&v)[kStepPieces], u32 acc) {
  const u64 wend = c.Pa - (u64)kStep * (c.S - 1 - i);
  const u64 r0 = wend - (u64)kStepRun * (lane_id() + 1);
  // keep payload bytes [s, pend) only; complement [s, s + 4) (the init value): only the top step
  // and the steps starting before s + 4 hold such pieces
  if (i + 1 == c.S || (int64_t)(wend - kStep) < (int64_t)(c.s + 4)) {
#pragma unroll
    for (int t = 0; t < kStepPieces; t++) {
      const u64 a = r0 + 16 * t;
      if (a < c.s + 4 || a + 16 > c.pend) {
        u64 klo, khi, xlo, xhi;
        range_mask((int)((int64_t)c.s - (int64_t)a), (int)((int64_t)c.pend - (int64_t)a), klo, khi);
        range_mask((int)((int64_t)c.s - (int64_t)a), (int)((int64_t)c.s + 4 - (int64_t)a), xlo, xhi);
        u64 lo = (u64)v[t].y << 32 | v[t].x, hi = (u64)v[t].w << 32 | v[t].z;
        lo = (lo & klo) ^ xlo;
        hi = (hi & khi) ^ xhi;
        v[t] = make_uint4((u32)lo, (u32)(lo >> 32), (u32)hi, (u32)(hi >> 32));
      }
    }
  }
  const u32 r = lane_id() & 31;
  u32 x = 0;
#pragma unroll
  for (int t = 0; t < kStepPieces; t++) {
    x = slice4(rep, r, x ^ v[t].x);
    x = slice4(rep, r, x ^ v[t].y);
    x = slice4(rep, r, x ^ v[t].z);
    x = slice4(rep, r, x ^ v[t].w);
  }
  // acc shifted by one step: four byte-table lookups instead of a 32-step GF(2) multiply
  const u32* sh = rep + kCrcRepWords + kWaves * kWaveLds / 4;
  const u32 t = xor3(sh[acc & 0xFF], sh[256 + ((acc >> 8) & 0xFF)], sh[512 + ((acc >> 16) & 0xFF)]) ^
                sh[768 + (acc >> 24)];
  return i == 0 ? x : (t ^ x);
}

// The list entries [lo, hi) (this workgroup's share of the bigwave list), one block per wave:
// waves claim them one at a time from an LDS counter (*pool, starting at lo), so a CU's faster
// waves take more blocks (its waves do not run at one speed: tpz_decode.hip decode_wave_kernel).
// Returns the blocks the wave decoded.
// rare: the worklist pointers (spill list / count, big list / count) from LDS, read only on the
// paths that append to them; as kernel arguments they were hoisted into SGPRs kept live across
// the block loop (at its SGPR limit: the spills went to VGPR lanes).
typedef __attribute__((address_space(1))) u32 gu32;
__device__ __forceinline__ void append(u32* const* rare, int k, u32 b) {
  if (lane_id() == 0) {
    gu32* l = (gu32*)rare[k];
    l[__hip_atomic_fetch_add((gu32*)rare[k + 1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)] = b;
  }
}
__device__ __forceinline__ u32 bigwave_phase(const BWParams& p, uint8_t* lds, u32 lo, u32 cnt,
                                             u32* pool, u32* const* rare) {
  u32* rep = reinterpret_cast<u32*>(lds);
  for (int i = threadIdx.x; i < kCrcRepWords / 4; i += kThreads)
    reinterpret_cast<uint4*>(rep)[i] = reinterpret_cast<const uint4*>(p.rep)[i];
  {   // shift-by-one-step tables: byte j of the CRC, value b -> gf_mul(x^(8 kStep), b << 8 j)
    u32* sh = rep + kCrcRepWords + kWaves * kWaveLds / 4;
    for (int i = threadIdx.x; i < kShiftWords; i += kThreads)
      sh[i] = gf_mul(p.step_shift, (u32)(i & 255) << (8 * (i >> 8)));
  }
  __syncthreads();
  const u32 wid = uni(threadIdx.x >> 6), lane = lane_id();
  Seg* seg = reinterpret_cast<Seg*>(lds + kCrcRepWords * 4 + wid * kWaveLds);
  uint8_t* cmap = reinterpret_cast<uint8_t*>(seg + kSegs);   // kU maps of 64 chunk slots
  auto next_it = [&]() -> u32 {        // the next entry, or >= cnt: none left
    u32 t = 0;
    if (lane == 0) t = atomicAdd(pool, 1u);
    return uni(t);
  };
  u32 ndone = 0;

#ifdef TPZ_BW_STAMPS
  u64 st_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  BW_T0();
  // Block i's list entry and extents are loaded during block i - 1 (scalar loads), and its
  // header words (n, the offsets, the stored CRC and the tag) during block i - 1's CRC, so a
  // block's parse starts with two memory round trips (key, then value lengths) instead of six.
  // The wave holds the entries of its next two blocks.
  u32 it = next_it();
  if (it >= cnt) return 0;
  u32 itn = next_it();
  u32 b = uni(ld_uniform(p.list, it));
  u64 s = ld_uniform(p.ext, b), e = ld_uniform(p.ext, b + 1);
  u32 hw = hdr_load(p, s, e);
  u32 bn = uni(ld_uniform(p.list, itn < cnt ? itn : it));
  for (;;) {
    BW_ST(5);
    const u32 itn2 = itn < cnt ? next_it() : itn;
    const u32 bnn = uni(ld_uniform(p.list, itn2 < cnt ? itn2 : it));
    const u64 sn = ld_uniform(p.ext, bn), en = ld_uniform(p.ext, bn + 1);
    bool hw_issued = false;
    u32 hwn = 0;
    auto issue_next_header = [&]() {
      if (!hw_issued) hwn = hdr_load(p, sn, en);
      hw_issued = true;
    };
    [&]() {
      const u32 len = (u32)(e - s);                   // > 4336 (the wave path's limit)
      const uint8_t* blk = p.src + s;
      const u32 tag = readlane(hw, 63) >> 24;                                  // compress.rs:99
      if (tag == 0 || tag > 3) { put_meta(p, b, TPZ_BLOCK_BAD_TAG, 0, 0); return; }  // :44-53
      if (tag != 1) { put_meta(p, b, TPZ_BLOCK_UNSUPPORTED_CODEC, 0, 0); return; }
      const u32 P = len - 5;
      const u32 stored = __builtin_bswap32(readlane(hw, 62));                 // block.rs:51
      const u32 w0 = readlane(hw, 0);
      const u32 n = ((w0 & 0xFFu) << 8) | ((w0 >> 8) & 0xFFu);                  // block.rs:54
      if (n >= kWave) {                     // (the wave path routes only n < 64 here)
        append(rare, 2, b);
        return;
      }
      u32 st = TPZ_BLOCK_OK, bcnt = n;
      // offset i: BE u16 at block byte 2 + 2 i, in header word (2 + 2 i) / 4
      const u32 q = 2 + 2 * lane;
      const u32 ow = (u32)__builtin_amdgcn_ds_bpermute((int)((q >> 2) << 2), (int)hw);
      const u32 osh = (q & 3u) * 8;
      if (P < 2 + 2 * n) {                                                     // block.rs:54-59
        st = TPZ_BLOCK_MALFORMED;
        bcnt = 0;
      } else {
        // ---- parse: lane i = entry i (n <= 63)
        const u32 dbo = 2 + 2 * n, dl = P - 2 - 2 * n;   // entries region, block offsets
        const bool act = lane < n;
        u32 off = 0, kl = 0, vl = 0;
        bool ok = true;
        if (act) {
          off = (((ow >> osh) & 0xFFu) << 8) | ((ow >> (osh + 8)) & 0xFFu);    // iterator.rs:74
          ok = off + 2 <= dl;
          if (ok) { kl = be16_at(blk + dbo + off); ok = off + 4 + kl <= dl; }   // :77-81
          if (ok) { vl = be16_at(blk + dbo + off + 2 + kl); ok = off + 4 + kl + vl <= dl; }
          if (!ok) kl = vl = 0;
        }
        const bool bad = __ballot(act && !ok) != 0;
        const u32 ki = scan_incl(kl), vi = scan_incl(vl);
        const u32 ktot = readlane(ki, 63), vtot = readlane(vi, 63);
        const u32 vs = (ktot + 15) & ~15u;                                     // tpz_value_start
        const bool slots_fit = 6u * n <= len;
        // the {kend, vend} pairs, whole 128-byte lines (pairs past n are zero)
        uint2* ends_g = reinterpret_cast<uint2*>(p.ends) + ends_base(p.efirst, s, b);
        if (slots_fit && lane < (p.efirst ? n : (n + 15) & ~15u))
          ends_g[lane] = act ? make_uint2(ki, vi) : make_uint2(0, 0);
        if (bad || !slots_fit || (u64)vs + vtot > (u64)len + 2) {
          // entries out of range (TPZ_BLOCK_BAD_ENTRY), or entries that overlap or repeat: the
          // spill path decodes the block (CRC included)
          append(rare, 0, b);
          return;
        } else {
          BW_ST(0);
          // ---- entry table: non-empty keys, then non-empty values, in stream order, then two
          // sentinels; deltas relative to the copy descriptor, which starts 16..31 bytes before
          // the block (so a second piece shifted back by up to 15 bytes stays inside it)
          const u64 rb = (s >= 16 ? s - 16 : 0) & ~15ull;
          const u64 rlim = (p.src_bytes < e + 16 ? p.src_bytes : e + 16) - rb;
          const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
              (void*)(p.src + rb), (short)0, (int)(rlim < 0x7FFFFFF0ull ? rlim : 0x7FFFFFF0ull), 0x00020000);
          const int sa = (int)(s - rb);                // block byte 0 in the descriptor
          const u64 kmask = __ballot(kl != 0), vmask = __ballot(vl != 0);
          const u32 knz = __builtin_popcountll(kmask), nseg = knz + __builtin_popcountll(vmask);
          if (kl) seg[lanes_below(kmask)] = Seg{ki, sa + (int)(dbo + off + 2) - (int)(ki - kl)};
          if (vl) seg[knz + lanes_below(vmask)] = Seg{vs + vi, sa + (int)(dbo + off + 4 + kl) - (int)(vs + vi - vl)};
          if (lane < 2) seg[nseg + lane] = Seg{0xFFFFFFFFu, 0};
          wave_lds_sync();
          // ---- copy: groups of kU 1 KiB windows; group g + 1 is mapped and its loads issued
          // before group g is merged and stored
          const u32 tot = vs + vtot, npad = (((tot + 15) >> 4) + 7) & ~7u, nwin = (npad + 63) >> 6;
          const __amdgpu_buffer_rsrc_t ds = __builtin_amdgcn_make_buffer_rsrc(
              (void*)(p.data + slot_base(s, b)), (short)0, (int)(16 * npad), 0x00020000);
#ifdef TPZ_BW_NOCOPY
          if (npad) return;                          // timing build only
#endif
          // Iteration i: issue CRC step i's loads, map group i + 1 and issue its loads, merge and
          // store group i, fold CRC step i. The waits for group i's loads and for step i's loads
          // leave the later-issued loads in flight (vmcnt counts in issue order).
          const FusedCrc fc = fused_crc_init(p, s, P);
          const u32 G = (nwin + kU - 1) / kU, I = max(G, fc.S);
          Group ga = {}, gb = {};                      // (initialised: not carried across blocks)
          uint4 cv[kStepPieces];
          u32 acc = 0;
          u32 m0 = G ? map_group(0, 0, nseg, seg, cmap, rs, ga) : 0;
          BW_ST(1);
#if TPZ_BW_PIPE
          for (u32 i = 0; i < I; i += 2) {             // unrolled by two: no group copies
            if (i < fc.S) fused_crc_issue(fc, i, cv);
            if (i + 1 < G) m0 = map_group((i + 1) * kU, m0, nseg, seg, cmap, rs, gb);
            BW_ST(1);
            if (i < G) store_group(i * kU, tot, nseg, seg, rs, ds, ga);
            BW_ST(3);
            if (i < fc.S) acc = fused_crc_fold(fc, p, rep, i, cv, acc);
            BW_ST(4);
            if (i + 1 >= I) break;
            if (i + 1 < fc.S) fused_crc_issue(fc, i + 1, cv);
            if (i + 2 < G) m0 = map_group((i + 2) * kU, m0, nseg, seg, cmap, rs, ga);
            BW_ST(1);
            if (i + 1 < G) store_group((i + 1) * kU, tot, nseg, seg, rs, ds, gb);
            BW_ST(3);
            if (i + 1 < fc.S) acc = fused_crc_fold(fc, p, rep, i + 1, cv, acc);
            BW_ST(4);
          }
#else
          for (u32 i = 0; i < I; i++) {                // one group at a time
#ifndef TPZ_BW_NOCRC
            if (i < fc.S) fused_crc_issue(fc, i, cv);
#endif
            if (i < G && i > 0) m0 = map_group(i * kU, m0, nseg, seg, cmap, rs, ga);
            BW_ST(1);
#ifndef TPZ_BW_NOCRC
            if (i < fc.S) acc = fused_crc_fold(fc, p, rep, i, cv, acc);
#endif
            BW_ST(4);
            if (i < G) store_group(i * kU, tot, nseg, seg, rs, ds, ga);
            BW_ST(3);
          }
#endif
          issue_next_header();
          const u32 R = wave_xor(gf_mul(p.step_lane_shift[lane], acc));
          const u32 k = (u32)(fc.Pa - fc.pend);
#ifdef TPZ_BW_NOCRC
          const u32 crc = stored + 0 * R * k;          // timing build only
#else
          const u32 crc = (R == shift_small(p, ~stored, k)) ? stored : ~unshift_small(p, R, k);
#endif
          if (crc != stored) {                                                 // checksum.rs:17
            st = TPZ_BLOCK_CHECKSUM_MISMATCH;
            bcnt = 0;
          }
          put_meta(p, b, st, bcnt, crc);
          return;
        }
      }
      BW_ST(5);
      issue_next_header();                   // lands during this block's CRC
      // ---- CRC (blocks that are not copied: malformed ones)
#ifdef TPZ_BW_NOCRC
      const u32 crc = stored;                        // timing build only
#else
      const u32 R = block_crc(p, rep, s, P);
      const u32 k = (u32)(((s + P + 15) & ~15ull) - (s + P));
      const u32 crc = (R == shift_small(p, ~stored, k)) ? stored : ~unshift_small(p, R, k);
#endif
      if (crc != stored) {                                                     // checksum.rs:17
        st = TPZ_BLOCK_CHECKSUM_MISMATCH;
        bcnt = 0;
      }
      BW_ST(4);
      put_meta(p, b, st, bcnt, crc);
    }();
    issue_next_header();
    ndone++;
    if (itn >= cnt) break;
    it = itn;
    itn = itn2;
    b = bn;
    s = sn;
    e = en;
    hw = hwn;
    bn = bnn;
  }
#ifdef TPZ_BW_STAMPS
  if (lane == 0)
    for (int q = 0; q < 8; q++) atomicAdd(&g_bw_stamps[q], (unsigned long long)st_[q]);
#endif
  return ndone;
}

static u32 gf_mul_host(u32 a, u32 b) {
  u32 r = 0;
  for (int i = 0; i < 32; i++) {
    if (a & (0x80000000u >> i)) r ^= b;
    b = (b >> 1) ^ ((b & 1u) ? 0xEDB88320u : 0u);
  }
  return r;
}
static u32 x8n_host(u64 nbytes) {                            // x^(8 n) mod P, reflected
  u32 r = 0x80000000u, sq = 0x80000000u >> 8;         // x^8
  for (u64 d = nbytes; d; d >>= 1) {
    if (d & 1u) r = gf_mul_host(r, sq);
    sq = gf_mul_host(sq, sq);
  }
  return r;
}

#ifdef TPZ_BW_STAMPS
extern "C" int tpz_debug_bw_stamps(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bw_stamps), sizeof(g_bw_stamps)) != hipSuccess) return 1;
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_bw_stamps), z, sizeof(z)) != hipSuccess) return 1;
  }
  return 0;
}
#endif

static BWParams bigwave_params(const BigWaveLaunch& a) {
  BWParams p{};
  p.src = a.src;
  p.ext = a.ext;
  p.src_bytes = a.src_bytes;
  p.rep = a.rep;
  p.tab = a.crc_tables;
  p.list = a.list;
  p.data = a.data;
  p.ends = a.ends;
  p.count = a.count;
  p.status = a.status;
  p.crc = a.crc;
  p.spill_list = a.spill_list;
  p.spill_count = a.spill_count;
  p.big_list = a.big_list;
  p.big_count = a.big_count;
  p.efirst = a.efirst;
  static const struct Shifts {     // computed once (~10^5 GF(2) steps: not per launch)
    u32 lane[64], step_lane[64], step, win, half;
    Shifts() {
      for (int l = 0; l < 64; l++) lane[l] = x8n_host((u64)kRun * l);
      for (int l = 0; l < 64; l++) step_lane[l] = x8n_host((u64)kStepRun * l);
      step = x8n_host(kStep);
      win = x8n_host(kCrcWin);
      half = x8n_host(kRun / 2);
    }
  } sh;
  for (int l = 0; l < 64; l++) p.lane_shift[l] = sh.lane[l];
  for (int l = 0; l < 64; l++) p.step_lane_shift[l] = sh.step_lane[l];
  p.step_shift = sh.step;
  p.win_shift = sh.win;
  p.half_shift = sh.half;
  return p;
}

// The bigwave list's kernel (before decode_tail_kernel, tpz_decode.hip): one workgroup per CU.
// (Its own unit on purpose: compiled into tpz_decode.hip, the same loop code ran 10 % slower on
// the 64k config, profiles/r3/tail_merge.jsonl.)
__global__ __launch_bounds__(kThreads, 1) void decode_bigwave_kernel(BWParams p, u32* ctr) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
  __shared__ u32 pool;
  __shared__ u32* rare[4];
  const u32 na = uni(tail_load(ctr + kTailBw));
  // this workgroup's share of the list: entries [lo, hi)
  const u32 per = (na + gridDim.x - 1) / gridDim.x, lo = blockIdx.x * per;
  const u32 hi = lo + per < na ? lo + per : na;
  if (lo >= hi) return;                              // an empty list costs one load
  if (threadIdx.x == 0) {                            // (the table upload's barrier publishes them)
    pool = lo;
    rare[0] = p.spill_list;
    rare[1] = p.spill_count;
    rare[2] = p.big_list;
    rare[3] = p.big_count;
  }
  bigwave_phase(p, lds, lo, hi, &pool, rare);
}

}  // namespace bw

void launch_bigwave(const BigWaveLaunch& a, uint32_t* ctr, uint32_t grid, hipStream_t stream) {
  hipLaunchKernelGGL(bw::decode_bigwave_kernel, dim3(grid), dim3(bw::kThreads), 0, stream,
                     bw::bigwave_params(a), ctr);
}

}  // namespace tpz
