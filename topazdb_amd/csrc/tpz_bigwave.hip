// tpz_bigwave.hip — gfx950 kernel for long blocks with few entries (the 64 KiB config:
// block_size 65536, 61 entries of 32-B keys and 1 KiB values), one wavefront per block.
//
// The LDS big path (decode_big_kernel) stages a whole block in a 92 KiB window, so a CU holds one
// block at a time and its CRC, parse and copy run back to back with the next block's bytes only in
// flight: 0.31 of the HBM roofline on the 64k config, 0.35 for its memory skeleton alone. Here
// nothing is staged. Each wave of a 16-wave workgroup decodes its own block straight from HBM,
// so a CU keeps 16 blocks in flight:
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

namespace tpz {

namespace {

typedef uint32_t u32;
typedef uint64_t u64;

constexpr int kWave = 64;
constexpr int kWaves = 16;
constexpr int kThreads = kWave * kWaves;
constexpr u32 kRun = 128;                         // CRC bytes per lane per window
constexpr u32 kCrcWin = kRun * kWave;             // 8 KiB
constexpr int kSegs = 128;                        // entry-table slots per wave (2 n <= 126)
constexpr int kU = 4;                             // copy windows in flight per wave
constexpr int kWaveLds = kSegs * 8 + kU * kWave * 4;   // entry table + kU u32 chunk maps
constexpr int kLdsBytes = kCrcRepWords * 4 + kWaves * kWaveLds;
static_assert(kLdsBytes <= 163840, "bigwave LDS");
constexpr u32 kOob = 0x80000000u;

__device__ __forceinline__ u32 lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
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
  const u32* list_count;
  uint8_t* data;
  u32* ends;
  u32* count;
  uint8_t* status;
  u32* crc;
  u32* spill_list;
  u32* spill_count;
  u32* big_list;
  u32* big_count;
  u32 lane_shift[64];       // x^(8 * 128 l) mod P
  u32 win_shift;            // x^(8 * 8192) mod P
  u32 half_shift;           // x^(8 * 64) mod P
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
    const u64 r0 = wend - (u64)kRun * (lane + 1);         // this lane's run [r0, r0 + 128)
    uint4 v[8];
#pragma unroll
    for (int t = 0; t < 8; t++) {
      const u64 a = r0 + 16 * t;
      v[t] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                           rs, (int64_t)a >= (int64_t)base ? (u32)(a - base) : kOob, 0, 0));
    }
    // keep payload bytes [s, pend) only; complement bytes [s, s + 4) (the init value)
#pragma unroll
    for (int t = 0; t < 8; t++) {
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
    // two independent chains (the run's halves) halve the lookup latency chain; the first half
    // is shifted past the second with x^(8*64)
    u32 ca = 0, cb = 0;
    const u32 r = lane & 31;
#pragma unroll
    for (int t = 0; t < 4; t++) {
      ca = slice4(rep, r, ca ^ v[t].x);
      cb = slice4(rep, r, cb ^ v[t + 4].x);
      ca = slice4(rep, r, ca ^ v[t].y);
      cb = slice4(rep, r, cb ^ v[t + 4].y);
      ca = slice4(rep, r, ca ^ v[t].z);
      cb = slice4(rep, r, cb ^ v[t + 4].z);
      ca = slice4(rep, r, ca ^ v[t].w);
      cb = slice4(rep, r, cb ^ v[t + 4].w);
    }
    const u32 c = gf_mul(p.half_shift, ca) ^ cb;
    const u32 part = wave_xor(gf_mul(ls, c));
    acc = (wi + 1 == W) ? part : (gf_mul(p.win_shift, acc) ^ part);
  }
  return acc;
}

// The 16 block bytes at block offset a (any int: a chunk's bytes are the segment's source
// shifted by the chunk's start, which can lie up to 15 bytes before the block when a short
// block's first entry starts near byte 0; those leading bytes read as zero).
__device__ __forceinline__ uint4 seg_load(__amdgpu_buffer_rsrc_t rs, u32 sa, int a, bool on) {
  const int c = a < 0 ? 0 : a;
  const uint4 v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                rs, on ? sa + (u32)c : kOob, 0, 0));
  if (a >= 0) return v;
  const u32 sh = (u32)(-a) * 8;                       // 8..120 bits
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

struct Seg {
  u32 end;      // exclusive end in the output stream
  int delta;    // (offset of its first byte in the block) - (its start in the stream)
};

__global__ __launch_bounds__(kThreads, 1) void decode_bigwave_kernel(BWParams p) {
  const u32 cnt = uni(*p.list_count);
  if (blockIdx.x * kWaves >= cnt) return;           // an empty list costs one load
  __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
  u32* rep = reinterpret_cast<u32*>(lds);
  for (int i = threadIdx.x; i < kCrcRepWords / 4; i += kThreads)
    reinterpret_cast<uint4*>(rep)[i] = reinterpret_cast<const uint4*>(p.rep)[i];
  __syncthreads();
  const u32 wid = uni(threadIdx.x >> 6), lane = lane_id();
  Seg* seg = reinterpret_cast<Seg*>(lds + kCrcRepWords * 4 + wid * kWaveLds);
  u32* cmap = reinterpret_cast<u32*>(seg + kSegs);   // kU maps of 64 chunk slots

#ifdef TPZ_BW_STAMPS
  u64 st_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  BW_T0();
  for (u32 it = blockIdx.x * kWaves + wid; it < cnt; it += gridDim.x * kWaves) {
    BW_ST(5);
    const u32 b = uni(p.list[it]);
    const u64 s = p.ext[b], e = p.ext[b + 1];
    const u32 len = (u32)(e - s);                     // > 4336 (the wave path's limit)
    const uint8_t* blk = p.src + s;
    const u32 tag = blk[len - 1];                                              // compress.rs:99
    if (tag == 0 || tag > 3) { put_meta(p, b, TPZ_BLOCK_BAD_TAG, 0, 0); continue; }  // :44-53
    if (tag != 1) { put_meta(p, b, TPZ_BLOCK_UNSUPPORTED_CODEC, 0, 0); continue; }
    const u32 P = len - 5;
    const u32 stored = ((u32)blk[P] << 24) | ((u32)blk[P + 1] << 16) | ((u32)blk[P + 2] << 8) |
                       blk[P + 3];                                             // block.rs:51
    const u32 n = be16_at(blk);                                                // block.rs:54
    if (n >= kWave) {                       // (the wave path routes only n < 64 here)
      if (lane == 0) p.big_list[atomicAdd(p.big_count, 1u)] = b;
      continue;
    }
    u32 st = TPZ_BLOCK_OK, bcnt = n;
    if (P < 2 + 2 * n) {                                                       // block.rs:54-59
      st = TPZ_BLOCK_MALFORMED;
      bcnt = 0;
    } else {
      // ---- parse: lane i = entry i (n <= 63)
      const u32 dbo = 2 + 2 * n, dl = P - 2 - 2 * n;   // entries region, block offsets
      const bool act = lane < n;
      u32 off = 0, kl = 0, vl = 0;
      bool ok = true;
      if (act) {
        off = be16_at(blk + 2 + 2 * lane);                                     // iterator.rs:74
        ok = off + 2 <= dl;
        if (ok) { kl = be16_at(blk + dbo + off); ok = off + 4 + kl <= dl; }     // :77-81
        if (ok) { vl = be16_at(blk + dbo + off + 2 + kl); ok = off + 4 + kl + vl <= dl; }
        if (!ok) kl = vl = 0;
      }
      const bool bad = __ballot(act && !ok) != 0;
      const u32 ki = scan_incl(kl), vi = scan_incl(vl);
      const u32 ktot = readlane(ki, 63), vtot = readlane(vi, 63);
      const u32 vs = (ktot + 15) & ~15u;                                       // tpz_value_start
      const bool slots_fit = 6u * n <= len;
      // the {kend, vend} pairs, whole 128-byte lines (pairs past n are zero)
      uint2* ends_g = reinterpret_cast<uint2*>(p.ends) + entry_base(s, b);
      if (slots_fit && lane < ((n + 15) & ~15u)) ends_g[lane] = act ? make_uint2(ki, vi) : make_uint2(0, 0);
      if (bad) {
        st = TPZ_BLOCK_MALFORMED;
        bcnt = 0;
      } else if (!slots_fit || (u64)vs + vtot > (u64)len + 2) {
        // entries overlap or repeat: the spill path decodes the block (CRC included)
        if (lane == 0) p.spill_list[atomicAdd(p.spill_count, 1u)] = b;
        continue;
      } else {
        BW_ST(0);
        // ---- entry table: non-empty keys, then non-empty values, in stream order
        const u64 kmask = __ballot(kl != 0), vmask = __ballot(vl != 0);
        const u32 knz = __builtin_popcountll(kmask), nseg = knz + __builtin_popcountll(vmask);
        if (kl) seg[lanes_below(kmask)] = Seg{ki, (int)(dbo + off + 2) - (int)(ki - kl)};
        if (vl) seg[knz + lanes_below(vmask)] = Seg{vs + vi, (int)(dbo + off + 4 + kl) - (int)(vs + vi - vl)};
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // ---- copy, 1 KiB windows
        const u32 tot = vs + vtot, nch = (tot + 15) >> 4, npad = (nch + 7) & ~7u;
        uint8_t* dst = p.data + slot_base(s, b);
        const u64 rb = s & ~15ull;                     // the block's bytes through a descriptor
        const u64 rlim = (p.src_bytes < e + 16 ? p.src_bytes : e + 16) - rb;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(p.src + rb), (short)0, (int)(rlim < 0x7FFFFFF0ull ? rlim : 0x7FFFFFF0ull), 0x00020000);
        const u32 sa = (u32)(s - rb);                  // block byte 0 in the descriptor
        // kU windows at a time. Their chunk maps are built together: segment k ending in chunk
        // slot t = ceil(end / 16) of window u sets map_u[t - 64 w] = max(., k + 1) (an LDS atomic
        // max: two segments ending in one chunk leave the larger index), then a prefix max per
        // window names the segment holding each chunk's start; every window's loads are issued
        // before any is used, so a wave has kU windows of loads in flight.
        u32 carry = 0;                                 // segments ending at or before w0's start
#ifdef TPZ_BW_NOCOPY
        if (npad) continue;                          // timing build only
#endif
        for (u32 w0 = 0; 64 * w0 < npad; w0 += kU) {
          u32 jv[kU], e0v[kU];
          uint4 av[kU], nv[kU];
          bool more = false;                           // a chunk meets 3+ segments
#pragma unroll
          for (int u = 0; u < kU; u++) cmap[u * kWave + lane] = 0;
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          u32 cu[kU];                                  // segments ending at or before window u
#pragma unroll
          for (int u = 0; u < kU; u++) cu[u] = carry;
          const u32 bend = 1024 * (w0 + kU);
          for (u32 k0 = carry; k0 < nseg; k0 += kWave) {
            const u32 k = k0 + lane;
            const u32 end = k < nseg ? seg[k].end : 0xFFFFFFFFu;
            const u32 t = (end + 15) >> 4;
            if (k < nseg && t >= 64 * w0 && t < 64 * (w0 + kU))
              atomicMax(&cmap[t - 64 * w0], k + 1);
#pragma unroll
            for (int u = 1; u < kU; u++)
              cu[u] += __builtin_popcountll(__ballot(k < nseg && end <= 1024 * (w0 + u)));
            if (readlane(end, 63) >= bend || k0 + kWave >= nseg) break;
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          u32 mv[kU];
#pragma unroll
          for (int u = 0; u < kU; u++) mv[u] = cmap[u * kWave + lane];
#pragma unroll
          for (int u = 0; u < kU; u++) {
            const u32 w = w0 + u;
            const u32 x0 = 1024 * w + 16 * lane, c = 64 * w + lane;
            const bool live = c < nch;
            u32 j = max(scan_max(mv[u]), cu[u]);
            Seg g0 = seg[j < nseg ? j : nseg - 1];
            while (live && j + 1 < nseg && g0.end <= x0) {   // (cannot happen: kept as a guard)
              j++;
              g0 = seg[j];
            }
            const bool two = live && j + 1 < nseg && g0.end < x0 + 16;
            const Seg g1 = seg[two ? j + 1 : j];
            more |= __ballot(two && g1.end < x0 + 16 && j + 2 < nseg) != 0;
            av[u] = seg_load(rs, sa, (int)x0 + g0.delta, live);
            nv[u] = seg_load(rs, sa, (int)x0 + g1.delta, two);
            jv[u] = j;
            e0v[u] = two ? g0.end : 0xFFFFFFFFu;
            if (u == kU - 1) carry = readlane(j, 63);
          }
          BW_ST(1);
#pragma unroll
          for (int u = 0; u < kU; u++) {
            const u32 w = w0 + u;
            const u32 x0 = 1024 * w + 16 * lane, c = 64 * w + lane;
            const bool live = c < nch;
            uint4 acc = av[u];
            u64 lo = (u64)acc.y << 32 | acc.x, hi = (u64)acc.w << 32 | acc.z;
            if (e0v[u] != 0xFFFFFFFFu) {               // the next segment's bytes after e0
              u64 mlo, mhi;
              range_mask((int)(e0v[u] - x0), 16, mlo, mhi);
              const u64 nlo = (u64)nv[u].y << 32 | nv[u].x, nhi = (u64)nv[u].w << 32 | nv[u].z;
              lo = (lo & ~mlo) | (nlo & mlo);
              hi = (hi & ~mhi) | (nhi & mhi);
            }
            if (more && live && e0v[u] != 0xFFFFFFFFu) {
              // chunks meeting 3+ segments (segments under 16 B): the rest one by one
              u32 jj = jv[u] + 1, eprev = seg[jj].end;
              while (jj + 1 < nseg && eprev < x0 + 16) {
                jj++;
                const Seg g = seg[jj];
                const uint4 nx = seg_load(rs, sa, (int)x0 + g.delta, true);
                u64 mlo, mhi;
                range_mask((int)(eprev - x0), 16, mlo, mhi);
                const u64 nlo = (u64)nx.y << 32 | nx.x, nhi = (u64)nx.w << 32 | nx.z;
                lo = (lo & ~mlo) | (nlo & mlo);
                hi = (hi & ~mhi) | (nhi & mhi);
                eprev = g.end;
              }
            }
            // bytes past the stream are zero; pad chunks up to the 128-byte line are zero
            u64 klo, khi;
            range_mask(0, live ? (int)min(tot - x0, 16u) : 0, klo, khi);
            lo &= klo;
            hi &= khi;
            if (c < npad)
              *reinterpret_cast<uint4*>(dst + x0) = make_uint4((u32)lo, (u32)(lo >> 32), (u32)hi, (u32)(hi >> 32));
          }
          BW_ST(3);
        }
      }
    }
    BW_ST(5);
    // ---- CRC
#ifdef TPZ_BW_NOCRC
    const u32 crc = stored;                        // timing build only
#else
    const u32 R = block_crc(p, rep, s, P);
    const u32 k = (u32)(((s + P + 15) & ~15ull) - (s + P));
    const u32 crc = (R == shift_small(p, ~stored, k)) ? stored : ~unshift_small(p, R, k);
#endif
    if (crc != stored) {                                                       // checksum.rs:17
      st = TPZ_BLOCK_CHECKSUM_MISMATCH;
      bcnt = 0;
    }
    BW_ST(4);
    put_meta(p, b, st, bcnt, crc);
  }
#ifdef TPZ_BW_STAMPS
  if (lane == 0)
    for (int q = 0; q < 8; q++) atomicAdd(&g_bw_stamps[q], (unsigned long long)st_[q]);
#endif
}

u32 gf_mul_host(u32 a, u32 b) {
  u32 r = 0;
  for (int i = 0; i < 32; i++) {
    if (a & (0x80000000u >> i)) r ^= b;
    b = (b >> 1) ^ ((b & 1u) ? 0xEDB88320u : 0u);
  }
  return r;
}
u32 x8n_host(u64 nbytes) {                            // x^(8 n) mod P, reflected
  u32 r = 0x80000000u, sq = 0x80000000u >> 8;         // x^8
  for (u64 d = nbytes; d; d >>= 1) {
    if (d & 1u) r = gf_mul_host(r, sq);
    sq = gf_mul_host(sq, sq);
  }
  return r;
}

}  // namespace

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

void launch_bigwave(const BigWaveLaunch& a, hipStream_t stream) {
  BWParams p{};
  p.src = a.src;
  p.ext = a.ext;
  p.src_bytes = a.src_bytes;
  p.rep = a.rep;
  p.tab = a.crc_tables;
  p.list = a.list;
  p.list_count = a.list_count;
  p.data = a.data;
  p.ends = a.ends;
  p.count = a.count;
  p.status = a.status;
  p.crc = a.crc;
  p.spill_list = a.spill_list;
  p.spill_count = a.spill_count;
  p.big_list = a.big_list;
  p.big_count = a.big_count;
  for (int l = 0; l < 64; l++) p.lane_shift[l] = x8n_host((u64)kRun * l);
  p.win_shift = x8n_host(kCrcWin);
  p.half_shift = x8n_host(kRun / 2);
  hipLaunchKernelGGL(decode_bigwave_kernel, dim3(a.grid), dim3(kThreads), 0, stream, p);
}

}  // namespace tpz
