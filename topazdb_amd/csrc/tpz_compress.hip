// tpz_compress.hip — compaction output with a codec on the device (Snappy, the default, or Lz4):
// compress::encode(data, CompressOptions::Snappy) (src/block/compress.rs:66-71, 82-93) for every
// Uncompress block of a batch the write side produced (tpz_encode_blocks): the payload and CRC
// (block.rs:31-44) become a snappy raw stream (snap::raw::Encoder::compress_vec's format: varint
// length, literal and copy elements), followed by tag 2. Blocks with another tag are copied
// unchanged (as the codec step copies non-compressed blocks).
//
// The snap crate's encoder is not in this image, so its output cannot be matched byte for byte:
// the stream here is a valid snappy stream of the same bytes (tests decode it with the oracle's
// snappy decoder and the device codec step, and hold it to the reference's ratio test,
// compress.rs:135-153). The match finder is snappy's (a 4-byte hash, the most recent earlier
// position per bucket, greedy), run by one wave per block over 64 positions at a time:
//   1. the lanes hash positions p .. p + 63 of the block (staged in LDS) and read their bucket:
//      a candidate from an earlier 64-position window, verified on its 4 bytes;
//   2. the first lane with a match (ballot) takes it; the lanes before it insert their positions
//      (a window without a match inserts all 64 and moves on);
//   3. the match is extended 64 bytes per round (ballot of the first mismatch), and the pending
//      literal and the copy are emitted (lane 0 writes headers, the wave copies literal bytes).
// Outputs go to a scratch slot per block (a closed-form bound of the encoded length, so blocks
// need no prefix pass first), then the sizes are scanned and the blocks packed back to back.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tpz_internal.h"

namespace tpz {
namespace {

typedef uint32_t u32;
typedef uint64_t u64;

constexpr int kCWaves = 16;
constexpr int kCWin = 4352;                 // staged block bytes: a0 (<= 15) + payload
constexpr u32 kCMaxStaged = kCWin - 16;     // longer payloads: literal-only stream
constexpr int kHashBits = 10;
constexpr int kCSlot = kCWin + (4 << kHashBits);

__device__ __forceinline__ u32 lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
__device__ __forceinline__ u32 uni(u32 x) { return __builtin_amdgcn_readfirstlane(x); }

// Unaligned little-endian u32 from an LDS byte array with a 4-aligned base.
__device__ __forceinline__ u32 ld4(const uint8_t* base, u32 a) {
  const u32* p = reinterpret_cast<const u32*>(base + (a & ~3u));
  return __builtin_amdgcn_alignbyte(p[1], p[0], a & 3u);
}

// Snappy elements (snap::raw's format): a varint preamble, literals (tag 00, the length - 1
// inline below 60, else in 1..4 bytes), copy-1 for 4..11 bytes within 2 KiB, else copy-2
// (1..64 bytes, a 2-byte offset); a long match is cut into pieces of at most 64 (never leaving
// a piece under 4).
struct SnappyEmit {
  static constexpr u32 kTag = 2;           // CompressOptions::Snappy
  uint8_t* out;   // the block's scratch slot
  u64 op;         // bytes written (wave-uniform)

  __device__ __forceinline__ void byte(u64 at, u32 v) const {
    if (lane_id() == 0) out[at] = (uint8_t)v;
  }
  __device__ __forceinline__ void begin(u64 m) {
    for (u64 v = m;; v >>= 7) {
      byte(op++, (u32)((v & 0x7F) | (v > 0x7F ? 0x80 : 0)));
      if (v <= 0x7F) break;
    }
  }
  // literal bytes src[lo .. hi) (LDS or global), at most 2^32 per element
  __device__ __forceinline__ void literal(const uint8_t* src, u64 lo, u64 hi) {
    if (hi <= lo) return;
    const u64 v = hi - lo - 1;
    u32 hl = 1;
    if (v < 60) {
      byte(op, (u32)v << 2);
    } else {
      const u32 nb = v < (1u << 8) ? 1u : v < (1u << 16) ? 2u : v < (1u << 24) ? 3u : 4u;
      byte(op, (59u + nb) << 2);
      for (u32 k = 0; k < nb; k++) byte(op + 1 + k, (u32)(v >> (8 * k)));
      hl = 1 + nb;
    }
    const u64 n = hi - lo;
    for (u64 i = lane_id(); i < n; i += 64) out[op + hl + i] = src[lo + i];
    op += hl + n;
  }
  __device__ __forceinline__ void copy(u32 off, u32 len) {
    while (len) {
      const u32 l = len > 64 ? (len - 64 < 4 ? 60u : 64u) : len;
      if (l >= 4 && l <= 11 && off < 2048) {
        byte(op, 1u | ((l - 4) << 2) | ((off >> 8) << 5));
        byte(op + 1, off & 0xFFu);
        op += 2;
      } else {
        byte(op, 2u | ((l - 1) << 2));
        byte(op + 1, off & 0xFFu);
        byte(op + 2, off >> 8);
        op += 3;
      }
      len -= l;
    }
  }
  __device__ __forceinline__ void seq(const uint8_t* src, u32 lo, u32 hi, u32 off, u32 len) {
    literal(src, lo, hi);
    copy(off, len);
  }
  __device__ __forceinline__ void last(const uint8_t* src, u64 lo, u64 hi) {
    for (; hi - lo > (1ull << 32); lo += 1ull << 32) literal(src, lo, lo + (1ull << 32));
    literal(src, lo, hi);
  }
  // matches start at q + 4 <= n and may run to the end
  static __device__ __forceinline__ u32 last_start(u32 n) { return n - 4; }
  static __device__ __forceinline__ u32 match_end(u32 n) { return n; }
};

// LZ4 block format as lz4::block::compress(data, None, true) writes it (compress.rs:73-77): the
// i32 LE size, then sequences: token (literal length | match length - 4, 15 = continued in
// 255-bytes), literals, a 2-byte LE offset, the match length continuation; the last sequence is
// literals only. The end rules LZ4_decompress_safe enforces (liblz4 1.9.3, oracle/tpz_lz4.c): a
// match starts at least 12 bytes before the end and ends at least 5 before it.
struct Lz4Emit {
  static constexpr u32 kTag = 3;           // CompressOptions::Lz4
  uint8_t* out;
  u64 op;

  __device__ __forceinline__ void byte(u64 at, u32 v) const {
    if (lane_id() == 0) out[at] = (uint8_t)v;
  }
  __device__ __forceinline__ void begin(u64 m) {
    for (int k = 0; k < 4; k++) byte(op + k, (u32)(m >> (8 * k)));
    op += 4;
  }
  __device__ __forceinline__ void length(u64 v) {      // a 15-continued length: 255s, remainder
    for (; v >= 255; v -= 255) byte(op++, 255);
    byte(op++, (u32)v);
  }
  __device__ __forceinline__ void literals(const uint8_t* src, u64 lo, u64 n) {
    for (u64 i = lane_id(); i < n; i += 64) out[op + i] = src[lo + i];
    op += n;
  }
  __device__ __forceinline__ void seq(const uint8_t* src, u32 lo, u32 hi, u32 off, u32 len) {
    const u32 ll = hi - lo, ml = len - 4;
    byte(op++, ((ll < 15 ? ll : 15u) << 4) | (ml < 15 ? ml : 15u));
    if (ll >= 15) length(ll - 15);
    literals(src, lo, ll);
    byte(op, off & 0xFFu);
    byte(op + 1, off >> 8);
    op += 2;
    if (ml >= 15) length(ml - 15);
  }
  __device__ __forceinline__ void last(const uint8_t* src, u64 lo, u64 hi) {
    const u64 ll = hi - lo;
    byte(op++, (ll < 15 ? (u32)ll : 15u) << 4);
    if (ll >= 15) length(ll - 15);
    literals(src, lo, ll);
  }
  // MFLIMIT (12) and LASTLITERALS (5)
  static __device__ __forceinline__ u32 last_start(u32 n) { return n >= 12 ? n - 12 : 0u; }
  static __device__ __forceinline__ u32 match_end(u32 n) { return n >= 5 ? n - 5 : 0u; }
};

struct CompressParams {
  const uint8_t* src;
  const u64* ext;
  u64 src_bytes;
  u32 n_blocks;
  uint8_t* scratch;
  u64* size;          // n_blocks + 1: each block's encoded length (scanned in place afterwards)
};

// The scratch slot of block i: ext[i] + ext[i] / 6 + 40 i. A block of L bytes encodes to at most
// 32 + L + L / 6 + 1 bytes (snappy's bound, the tag), and consecutive slots are at least
// L + L / 6 + 40 apart.
__device__ __host__ __forceinline__ u64 cslot(u64 ext_i, u64 i) { return ext_i + ext_i / 6 + 40 * i; }

template <class Emit>
__global__ __launch_bounds__(1024) void compress_kernel(CompressParams p) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kCWaves * kCSlot];
  const u32 lane = lane_id(), wid = uni(threadIdx.x >> 6);
  uint8_t* win = lds + wid * kCSlot;
  u32* tab = reinterpret_cast<u32*>(win + kCWin);
  const u32 nw = gridDim.x * kCWaves;
  for (u32 b = blockIdx.x * kCWaves + wid; b < p.n_blocks; b += nw) {
    const u64 s = p.ext[b], e = p.ext[b + 1], L = e - s;
    uint8_t* out = p.scratch + cslot(s, b);
    const u32 tag = L ? p.src[e - 1] : 0u;
    if (L == 0 || tag != 1) {                         // not an Uncompress block: unchanged
      for (u64 i = lane; i < L; i += 64) out[i] = p.src[s + i];
      if (lane == 0) p.size[b] = L;
      continue;
    }
    const u64 m = L - 1;                              // payload | crc: the bytes the codec sees
    Emit E{out, 0};
    E.begin(m);
    if (m > kCMaxStaged) {
      // past the LDS window: one literal run straight from HBM (a valid stream, uncompressed)
      E.last(p.src + s, 0, m);
      E.byte(E.op, Emit::kTag);
      if (lane == 0) p.size[b] = E.op + 1;
      continue;
    }
    // stage [s & ~15, s + m) (16-byte loads; bytes past the block are never used)
    const u32 a0 = (u32)(s & 15u);
    {
      const u64 ws = s & ~15ull;
      const u32 nbytes = (u32)(s + m - ws);
      for (u32 o = 16 * lane; o < nbytes; o += 1024) {
        uint4 v;
        if (ws + o + 16 <= p.src_bytes) {
          v = *reinterpret_cast<const uint4*>(p.src + ws + o);
        } else {
          u32 w[4] = {0, 0, 0, 0};
          for (u32 k = 0; k < 16; k++)
            if (ws + o + k < p.src_bytes) w[k >> 2] |= (u32)p.src[ws + o + k] << (8 * (k & 3));
          v = make_uint4(w[0], w[1], w[2], w[3]);
        }
        *reinterpret_cast<uint4*>(win + o) = v;
      }
      __builtin_amdgcn_wave_barrier();
    }
    const uint8_t* d = win + a0;
    const u32 n = (u32)m;
    const u32 qlast = Emit::last_start(n), mend = Emit::match_end(n);
    u32 pos = 0, lit = 0;
    while (n >= 4 && pos <= qlast) {
      const u32 q = pos + lane;
      const bool ok = q <= qlast;
      const u32 w = ok ? ld4(win, a0 + q) : 0u;
      const u32 h = (w * 0x1E35A7BDu) >> (32 - kHashBits);
      // a bucket holds a position of an earlier window of this block, or another block's: only a
      // verified candidate before q counts
      const u32 c = ok ? tab[h] : 0u;
      const bool hit = ok && c < pos && q - c < 65536 && q + 4 <= mend && ld4(win, a0 + c) == w;
      const u64 hm = __ballot(hit);
      if (!hm) {
        if (ok) tab[h] = q;
        pos += 64;
        continue;
      }
      const u32 f = (u32)__builtin_ctzll(hm);
      const u32 qf = pos + f, cf = __builtin_amdgcn_readlane(c, f);
      if (ok && lane <= f) tab[h] = q;
      // extend the match past its first 4 bytes, 64 bytes per round, up to mend
      u32 len = 4;
      for (;;) {
        const u32 k = qf + len + lane;
        const bool same = k < mend && d[k] == d[cf + len + lane];
        const u64 mm = ~__ballot(same);
        if (mm) {
          len += (u32)__builtin_ctzll(mm);
          break;
        }
        len += 64;
      }
      E.seq(d, lit, qf, qf - cf, len);
      pos = qf + len;
      lit = pos;
    }
    E.last(d, lit, n);
    E.byte(E.op, Emit::kTag);
    if (lane == 0) p.size[b] = E.op + 1;
  }
}

// Block i's encoded bytes from its scratch slot to dst[first[i] ..] (first = the scanned sizes):
// one wave per block, 16-byte chunks aligned to dst, the chunks shared with the neighbours
// written byte by byte.
__global__ __launch_bounds__(256) void compress_pack_kernel(const uint8_t* scratch, const u64* ext,
                                                            const u64* first, u32 n_blocks,
                                                            uint8_t* dst) {
  const u32 lane = lane_id();
  const u32 nw = gridDim.x * 4;
  for (u32 b = blockIdx.x * 4 + uni(threadIdx.x >> 6); b < n_blocks; b += nw) {
    const uint8_t* s = scratch + cslot(ext[b], b);
    const u64 d0 = first[b], len = first[b + 1] - d0;
    if (!len) continue;
    const u64 head = (16 - (d0 & 15)) & 15;                      // bytes before dst's first chunk
    const u64 h = head < len ? head : len;
    if (lane < h) dst[d0 + lane] = s[lane];
    const u64 body = (len - h) & ~15ull;
    for (u64 o = 16 * (u64)lane; o < body; o += 1024) {
      uint4 v;
      __builtin_memcpy(&v, s + h + o, 16);
      *reinterpret_cast<uint4*>(dst + d0 + h + o) = v;
    }
    const u64 t0 = h + body;
    if (lane < len - t0) dst[d0 + t0 + lane] = s[t0 + lane];
  }
}

}  // namespace

uint64_t compress_scratch_bytes(uint64_t src_bytes, uint32_t n_blocks) {
  return cslot(src_bytes, n_blocks) + 64;
}

void launch_compress(const uint8_t* src, const u64* ext, u64 src_bytes, u32 n_blocks, u32 codec,
                     uint8_t* scratch, u64* sizes, u64* part, uint8_t* dst, u32 num_cus,
                     hipStream_t stream) {
  if (n_blocks == 0) {
    (void)hipMemsetAsync(sizes, 0, 8, stream);
    return;
  }
  CompressParams p{src, ext, src_bytes, n_blocks, scratch, sizes};
  u32 grid = (n_blocks + kCWaves - 1) / kCWaves;
  if (grid > num_cus) grid = num_cus;      // 16 waves (132 KiB of LDS) per CU, persistent
  if (codec == 3)
    hipLaunchKernelGGL(compress_kernel<Lz4Emit>, dim3(grid), dim3(1024), 0, stream, p);
  else
    hipLaunchKernelGGL(compress_kernel<SnappyEmit>, dim3(grid), dim3(1024), 0, stream, p);
  launch_scan_u64(sizes, n_blocks, part, stream);
  u32 g2 = (n_blocks + 3) / 4;
  if (g2 > 8 * num_cus) g2 = 8 * num_cus;
  hipLaunchKernelGGL(compress_pack_kernel, dim3(g2), dim3(256), 0, stream, scratch, ext, sizes,
                     n_blocks, dst);
}

}  // namespace tpz
