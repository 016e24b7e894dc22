// tpz_codec.hip — gfx950 kernels for the block codec step of compress::decode
// (src/block/compress.rs:95-113): snappy (tag 2) blocks are decompressed on the device and
// re-tagged Uncompress (tag 1), so that tpz_decode_blocks then decodes them like any block.
//
// snappy raw format (the `snap` crate's decompress_vec, compress.rs:104-107; restated from the
// published format description, as oracle/tpz_snappy.c): a varint with the uncompressed length,
// then elements — literal (tag & 3 == 0: len-1 in tag >> 2, or in 1-4 little-endian bytes when
// tag >> 2 >= 60), copy-1 (len 4 + (tag >> 2 & 7), 11-bit offset), copy-2 (len 1 + (tag >> 2),
// 16-bit offset), copy-4 (32-bit offset). snap's Err cases (truncated varint or element, offset
// 0 or past the output, output over- or underrun) give TPZ_BLOCK_CODEC_ERROR.
//
// Execution: one wave per block. The compressed bytes are staged in LDS; the
// element headers are parsed with wave-uniform reads (one LDS round trip per element: the tag and
// its next 7 bytes); every element's bytes are produced by the 64 lanes in parallel (a copy whose
// offset is shorter than its length repeats with period `offset`, so lane k reads byte
// d - offset + k mod offset, which precedes the copy). The output is assembled in LDS and stored
// with 16-byte stores (byte stores at the two edge pieces, which neighbouring blocks share).
// Blocks larger than a 16-wave workgroup's slots go to a one-wave-per-workgroup kernel with
// 64 KiB input / 94 KiB output windows; blocks past those windows (no size limit: snap and lz4
// decode any length) are decompressed by that wave straight from HBM to HBM.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tpz_internal.h"

namespace tpz {

namespace {

typedef uint32_t u32;
typedef uint64_t u64;

constexpr int kWave = 64;
#ifndef TPZ_CODEC_WAVES
#define TPZ_CODEC_WAVES 16                           // diagnostic builds vary it
#endif
constexpr int kSmallWaves = TPZ_CODEC_WAVES;
constexpr u32 kSmallIn = 4608, kSmallOut = 5120;     // per-wave windows of the 16-wave kernel
constexpr u32 kBigIn = 65536, kBigOut = 94208;       // the one-wave kernel
constexpr u32 kGuard = 16;                           // readable bytes before each input window
constexpr u32 kInSlack = 16 + 16;                    // staging offset (< 16) + header overread
constexpr u64 kMaxInWindow = kBigIn - kInSlack;      // 65504: compressed bytes a window takes
constexpr uint8_t kLeftForWaveKernel = 0xFF;         // status the group pass leaves behind
static_assert(kSmallWaves * (kGuard + kSmallIn + kSmallOut) <= 163840, "small LDS");
static_assert(kGuard + kBigIn + kBigOut <= 163840, "big LDS");

#ifdef TPZ_CODEC_STAMPS
// Diagnostic build only (make -C topazdb_amd/csrc codec-variants): per-phase wave cycles.
__device__ unsigned long long g_cstamps[8];
struct Stamps {
  u64 acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  u64 t = __builtin_amdgcn_s_memtime();
  __device__ void hit(int i) {
    const u64 n = __builtin_amdgcn_s_memtime();
    acc[i] += n - t;
    t = n;
  }
  __device__ void add(int i, u64 v) { acc[i] += v; }
  __device__ void flush(bool lane0) {
    if (lane0)
      for (int i = 0; i < 8; i++) atomicAdd(&g_cstamps[i], (unsigned long long)acc[i]);
  }
};
#define STAMP(i) st_.hit(i)
#define SCOUNT(i, v) st_.add(i, v)
#define STAMPS_ARG , Stamps& st_
#define STAMPS_PASS , st_
#else
#define STAMP(i) (void)0
#define SCOUNT(i, v) (void)0
#define STAMPS_ARG
#define STAMPS_PASS
#endif

// an opaque VGPR copy: the compiler cannot prove the value wave-uniform, so the header decode and
// the positions derived from it stay on the VALU (branches on them become exec-masked regions
// that skip when empty)
__device__ __forceinline__ u32 vgpr_opaque(u32 x) {
  u32 y;
  asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "v"(x));
  return y;
}
#define CODEC_HDR(x) vgpr_opaque(x)

__device__ __forceinline__ u32 lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
__device__ __forceinline__ u32 uni(u32 x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ u64 uni64(u64 x) {
  const u32 lo = __builtin_amdgcn_readfirstlane((u32)x);
  const u32 hi = __builtin_amdgcn_readfirstlane((u32)(x >> 32));
  return ((u64)hi << 32) | lo;
}

// Little-endian u32 at any LDS byte address: two aligned reads + alignbyte. (Pointer arithmetic
// only, so the accesses stay ds_read: a round trip through an integer would make them flat.)
__device__ __forceinline__ u32 lds_u32_lane(const uint8_t* p) {
  const u32 al = (u32)reinterpret_cast<uintptr_t>(p) & 3u;
  const u32* q = reinterpret_cast<const u32*>(p - al);
  return __builtin_amdgcn_alignbyte(q[1], q[0], al);
}
// The same, wave-uniform.
__device__ __forceinline__ u32 lds_u32(const uint8_t* base, u32 a) {
  return uni(lds_u32_lane(base + a));
}

// Snappy varint preamble from global memory (at most 10 bytes, inside the block). Returns the
// header length, 0 if the varint is truncated or does not fit 32 bits (snap: Error::Header /
// TooBig).
__device__ __forceinline__ u32 snappy_header(const uint8_t* s, u64 n, u64& want) {
  u64 v = 0;
  for (u32 i = 0; i < 10 && i < n; i++) {
    const u32 c = s[i];
    v |= (u64)(c & 0x7F) << (7 * i);
    if (!(c & 0x80)) {
      if (v > 0xFFFFFFFFull) return 0;
      want = v;
      return i + 1;
    }
  }
  return 0;
}

struct CodecParams {
  const uint8_t* src;
  const u64* ext;
  u64 src_bytes;
  u32 n_blocks;
  uint8_t* dst;
  const u64* dst_ext;
  u64* size;         // sizes kernel output
  uint8_t* status;
  u32* defer_list;
  u32* defer_count;
  u32 group_pass;    // the lane kernels ran first (status 0xFF = left for the wave kernel)
  u32 claimed;       // sizes kernel: LZ4 blocks take their size prefix (tpz_decompressed_sizes_claimed)
  u32* inexact;      // decompress: sticky word, set when an LZ4 block's range is not its exact length
};

// ------------------------------------------------------------------ per-block work
// Copies LDS bytes to global [g, g + n). The bytes sit at win[(g & 15) ..], i.e. LDS and global
// share their alignment, so every whole 16-byte piece is one ds_read_b128 + one global store;
// the (shared) edge pieces take byte stores.
__device__ __forceinline__ void store_aligned(const uint8_t* win, uint8_t* g, u32 n) {
  const u32 lane = lane_id();
  if (n == 0) return;
  const u32 a = (u32)(reinterpret_cast<uintptr_t>(g) & 15);
  const u32 head = (16 - a) & 15;
  const u32 h = head < n ? head : n;
  const u32 body = (n - h) & ~15u;
  for (u32 k = lane; k < h; k += kWave) g[k] = win[a + k];
  for (u32 k = 16 * lane; k < body; k += 16 * kWave)
    *reinterpret_cast<uint4*>(g + h + k) = *reinterpret_cast<const uint4*>(win + a + h + k);
  for (u32 k = h + body + lane; k < n; k += kWave) g[k] = win[a + k];
}

// Stages global bytes [s, s + n) into LDS at win[(s & 15) ..]: 16-byte aligned loads, four
// 1 KiB rounds in flight per step (the bytes around the range are don't-care).
__device__ __forceinline__ void stage_aligned(const uint8_t* src, u64 src_bytes, u64 s, u32 n,
                                              uint8_t* win) {
  const u32 lane = lane_id();
  const u64 ws = s & ~15ull;
  const u32 nb = (u32)(s + n - ws);
  const u64 lim = src_bytes - ws < 0x7FFFFFF0ull ? src_bytes - ws : 0x7FFFFFF0ull;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(src + ws), (short)0, (int)lim, 0x00020000);
  for (u32 off = 0; off < nb; off += 4096) {
    uint4 t[4];
#pragma unroll
    for (int r = 0; r < 4; r++)
      t[r] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + r * 1024 + lane * 16, 0, 0));
#pragma unroll
    for (int r = 0; r < 4; r++)
      if (off + r * 1024 + lane * 16 < nb) *reinterpret_cast<uint4*>(win + off + r * 1024 + lane * 16) = t[r];
  }
  // a piece straddling the end of the buffer came back zeroed: refill its in-range bytes
  const u64 last = (s + n - 1) & ~15ull;
  if (last + 16 > src_bytes)
    for (u32 k = lane; k < 16; k += kWave)
      if (last + k < s + n) win[last - ws + k] = src[last + k];
}

// out[d .. d + len) = in[ip .. ip + len) in LDS. The bytes up to the next 4-byte boundary of
// the output are written one per lane; the rest as whole aligned dwords (two aligned input reads
// + alignbyte), the last of which may write up to 3 bytes past the literal: those bytes belong to
// later elements, whose writes come after in LDS order, and nothing reads past `d`.
__device__ __forceinline__ void literal_copy(const uint8_t* in, u32 ip, uint8_t* out, u32 d,
                                             u32 len) {
  const u32 lane = lane_id();
  const u32 pad0 = (0u - (u32)reinterpret_cast<uintptr_t>(out + d)) & 3u;
  const u32 pad = pad0 < len ? pad0 : len;
  if (lane < pad) out[d + lane] = in[ip + lane];
  const u32 nd = (len - pad + 3) >> 2;
  u32* o = reinterpret_cast<u32*>(out + d + pad);
  const uint8_t* i = in + ip + pad;
  for (u32 t = lane; t < nd; t += kWave) o[t] = lds_u32_lane(i + 4 * t);
}

// Decompresses the snappy stream in[0 .. n) (elements from `ip`) into out[0 .. want).
// Wave-uniform control flow, kept lean: the loop is bound by scalar issue (one SALU instruction
// per SIMD every 4 cycles, shared by the SIMD's waves), so the header is decoded with selects and
// every check folds into one branch. The next element's header is read before the current
// element's bytes are copied, so its LDS latency overlaps the copy (the input is never written).
__device__ __forceinline__ bool snappy_decode(const uint8_t* in, u32 n, u32 ip, uint8_t* out,
                                              u32 want STAMPS_ARG) {
  const u32 lane = lane_id();
  u32 d = 0;
  // the next header as three aligned dwords in VGPRs (+ its alignment): combined only at the top
  // of the next iteration
  u32 al = (u32)reinterpret_cast<uintptr_t>(in + ip) & 3u;
  const u32* q = reinterpret_cast<const u32*>(in + ip - al);
  u32 r0 = q[0], r1 = q[1], r2 = q[2];
  while (ip < n) {
    // the header stays in VGPRs (wave-uniform values): its decode then issues on the VALU and
    // only the branch conditions cross to the scalar unit (the loop is scalar-issue bound;
    // 2.77 vs 3.11 ms per 2^18 blocks with the header on the scalar unit, TPZ_CODEC_SALU)
    const u32 w0 = CODEC_HDR(__builtin_amdgcn_alignbyte(r1, r0, al));
    const u32 w1 = CODEC_HDR(__builtin_amdgcn_alignbyte(r2, r1, al));
    const u32 tag = w0 & 0xFF, kind = tag & 3, t6 = tag >> 2;
    const u32 x = (w0 >> 8) | (w1 << 24);                     // the 4 bytes after the tag
    // literal: length - 1 in t6, or in the next t6 - 59 bytes when t6 >= 60
    const u32 nb = t6 >= 60 ? t6 - 59 : 0u;
    u32 lx = nb == 0 ? t6 : (nb == 4 ? x : x & ((1u << (8 * nb)) - 1));
    lx = lx < 0x7FFFFFFFu ? lx : 0x7FFFFFFFu;                 // past any window: fails below
    const u32 len = kind == 0 ? lx + 1 : (kind == 1 ? 4 + (t6 & 7) : t6 + 1);
    const u32 hl = kind == 0 ? 1 + nb : (0x5320u >> (4 * kind)) & 15;
    const u32 off = kind == 1 ? ((tag >> 5) << 8) | (x & 0xFF) : (kind == 2 ? x & 0xFFFF : x);
    const u32 next = ip + hl + (kind == 0 ? len : 0u);
    // snap's Err: output overrun, element past the input, copy offset 0 or before the output
    if (d + len > want || next > n || (kind != 0 && off - 1 >= d)) return false;
    al = (u32)reinterpret_cast<uintptr_t>(in + next) & 3u;    // prefetch the next header
    q = reinterpret_cast<const u32*>(in + next - al);
    r0 = q[0];
    r1 = q[1];
    r2 = q[2];
    if (kind == 0) {
      literal_copy(in, ip + hl, out, d, len);
    } else if (lane < len) {
      // copies are at most 64 bytes: one byte per lane; an overlapping copy (off < len) repeats
      // with period off (lane % off from a float reciprocal: exact for lane, off <= 64)
      const u32 qq = (u32)(((float)lane + 0.5f) * __builtin_amdgcn_rcpf((float)off));
      const u32 r = off >= len ? lane : lane - qq * off;
      out[d + lane] = out[d - off + r];
    }
    ip = next;
    d += len;
    SCOUNT(6, 1);
  }
  return d == want;
}

// ------------------------------------------------------------------ LZ4 (codec 3)
// lz4::block::decompress(data, None) (src/block/compress.rs:108-111): i32 LE size prefix (Err if
// the source is shorter than 4 bytes, the size is negative or above LZ4_compressBound's limit
// 0x7E000000), then LZ4_decompress_safe(src + 4, dst, len - 4, size); the output is the `ret`
// bytes it decodes (possibly fewer than `size`). The acceptance rules below are liblz4 1.9.3's
// LZ4_decompress_generic for LZ4_decompress_safe, restated as oracle/tpz_lz4.c does (and pinned
// against liblz4 by tests/test_lz4_oracle.py): the fast loop while >= 64 output bytes remain,
// then the safe loop with its two-stage shortcut. A match repeats the bytes `offset` back
// (periodic when it overlaps); an offset-0 match is zeros. `Src` reads input bytes, `Out`
// copies (or not: the sizes pass only walks).
struct Lz4NoOut {
  __device__ void lit(int64_t, int64_t, int64_t) const {}
  __device__ void match(int64_t, int64_t, int64_t) const {}
};
struct Lz4GlobalSrc {            // per thread, straight from global memory
  const uint8_t* p;
  __device__ u32 byte(int64_t i) const { return p[i]; }
};
struct Lz4LdsSrc {               // wave-uniform, from the staged bytes
  const uint8_t* p;
  __device__ u32 byte(int64_t i) const { return uni(p[i]); }  // scalar: 17 % faster than VALU here
};

__device__ __forceinline__ void match_copy_wave(uint8_t* out, u32 d, u32 off, u32 len) {
  const u32 lane = lane_id();
  if (off == 0) {
    for (u32 k = lane; k < len; k += kWave) out[d + k] = 0;
  } else if (off >= (u32)kWave) {
    // each round of 64 bytes reads bytes at least 64 back: written by earlier rounds
    for (u32 k = lane; k < len; k += kWave) out[d + k] = out[d + k - off];
  } else {
    // period off: byte k is byte k mod off of the run before d
    u32 r = lane - (u32)(((float)lane + 0.5f) * __builtin_amdgcn_rcpf((float)off)) * off;
    const u32 c = (u32)kWave % off;
    for (u32 k = lane; k < len; k += kWave) {
      out[d + k] = out[d - off + r];
      r += c;
      r = r >= off ? r - off : r;
    }
  }
}

struct Lz4WaveOut {              // wave-wide copies into the LDS output window
  const uint8_t* in;
  uint8_t* out;
  __device__ void lit(int64_t op, int64_t ip, int64_t len) const {
    literal_copy(in, (u32)ip, out, (u32)op, (u32)len);
  }
  __device__ void match(int64_t op, int64_t off, int64_t len) const {
    match_copy_wave(out, (u32)op, (u32)off, (u32)len);
  }
};

typedef unsigned __int128 u128;

__device__ __forceinline__ u128 ld16u(const uint8_t* p) {    // unaligned 16-byte load
  u128 v;
  __builtin_memcpy(&v, p, 16);
  return v;
}
__device__ __forceinline__ void st16u(uint8_t* p, u128 v) { __builtin_memcpy(p, &v, 16); }

// 16 bytes at base[a ..] of a buffer of size >= 16 bytes: the load is clamped inside the buffer
// and the bytes past its end read as zero (branch-free, so the waits on a lane's loads stay exact)
__device__ __forceinline__ u128 ld16c(const uint8_t* base, u64 size, u64 a) {
  const u64 ac = a + 16 <= size ? a : size - 16;
  const u128 v = ld16u(base + ac);
  const u64 sh = a - ac;
  return sh == 0 ? v : (sh >= 16 ? (u128)0 : v >> (8 * sh));
}

// per thread through a 16-byte register window (one 16-byte load per window instead of a
// dependent byte load per header byte)
// cpos starts 2^62 before base, so the first byte read always loads a window (a start of ~0
// made the window look valid for addresses below 15, reading zeros)
struct Lz4LaneSrc {
  const uint8_t* src;
  u64 src_bytes, base;          // in[0] is src[base]
  mutable u64 cpos;
  mutable u128 cv;
  __device__ u32 byte(int64_t i) const {
    const u64 a = base + (u64)i;
    if (a - cpos >= 16) {
      cpos = a;
      cv = ld16c(src, src_bytes, a);
    }
    return (u32)(cv >> (8 * (a - cpos))) & 0xFFu;
  }
};
// the sizes pass's source: the lane's own 128-byte window in LDS, refilled at a 16-byte boundary
// with eight 16-byte loads. The walk is a chain of dependent loads: in the compressible 4 KiB
// shape a sequence is a ~70-byte literal and a match, so a 16-byte register window needed a
// load per sequence, while the next header after a literal of up to ~110 bytes is still in the
// 128-byte window (the byte reads become LDS round trips). 32 KiB per 256-thread workgroup, so
// five workgroups (20 waves) share a CU, as many as the kernel's VGPRs allow.
constexpr u32 kLz4WinStride = 128;
struct Lz4LaneWinSrc {
  const uint8_t* src;
  u64 src_bytes, base;          // in[0] is src[base]
  mutable u64 cpos;             // the window's first byte (starts 2^62 before base: no window)
  uint8_t* win;                 // this lane's window (LDS)
  __device__ u32 byte(int64_t i) const {
    const u64 a = base + (u64)i;
    if (a - cpos >= 128) {
      cpos = a & ~15ull;
      u128 v[8];
#pragma unroll
      for (int t = 0; t < 8; t++) v[t] = ld16c(src, src_bytes, cpos + 16 * t);
#pragma unroll
      for (int t = 0; t < 8; t++) {
        reinterpret_cast<uint64_t*>(win)[2 * t] = (uint64_t)v[t];
        reinterpret_cast<uint64_t*>(win)[2 * t + 1] = (uint64_t)(v[t] >> 64);
      }
    }
    return win[a - cpos];
  }
};
template <class Src, class Out>
__device__ int64_t lz4_walk(const Src& in, int64_t iend, const Out& out, int64_t oend) {
  if (oend == 0) return (iend == 1 && in.byte(0) == 0) ? 0 : -1;
  if (iend == 0) return -1;
  const int64_t shortiend = iend - 16, shortoend = oend - 32;
  int64_t ip = 0, op = 0, lit = 0, ml = 0, off = 0, match = 0, cpy = 0;
  u32 token = 0;
  if (oend >= 64) {
    for (;;) {                                                // fast loop
      token = in.byte(ip++);
      lit = token >> 4;
      if (lit == 15) {
        if (ip >= iend - 15) return -1;
        u32 sv;
        do {
          sv = in.byte(ip++);
          lit += sv;
          if (ip >= iend - 15) break;
        } while (sv == 255);
        cpy = op + lit;
        if (cpy > oend - 32 || ip + lit > iend - 32) goto safe_literal_copy;
      } else {
        cpy = op + lit;
        if (ip > iend - 17) goto safe_literal_copy;
      }
      out.lit(op, ip, lit);
      ip += lit;
      op = cpy;
      off = (int64_t)(in.byte(ip) | in.byte(ip + 1) << 8);
      ip += 2;
      match = op - off;
      ml = token & 15;
      if (ml == 15) {
        if (match < 0) return -1;
        u32 sv;
        do {
          sv = in.byte(ip++);
          ml += sv;
          if (ip >= iend - 4) return -1;
        } while (sv == 255);
        ml += 4;
        if (op + ml >= oend - 64) goto safe_match_copy;
      } else {
        ml += 4;
        if (op + ml >= oend - 64) goto safe_match_copy;
      }
      if (match < 0) return -1;
      out.match(op, off, ml);
      op += ml;
    }
  }
  for (;;) {                                                  // safe loop
    token = in.byte(ip++);
    lit = token >> 4;
    if (lit != 15 && ip < shortiend && op <= shortoend) {     // the shortcut
      out.lit(op, ip, lit);
      op += lit;
      ip += lit;
      ml = token & 15;
      off = (int64_t)(in.byte(ip) | in.byte(ip + 1) << 8);
      ip += 2;
      match = op - off;
      if (ml != 15 && off >= 8 && match >= 0) {
        out.match(op, off, ml + 4);
        op += ml + 4;
        continue;
      }
      goto copy_match;
    }
    if (lit == 15) {
      if (ip >= iend - 15) return -1;
      u32 sv;
      do {
        sv = in.byte(ip++);
        lit += sv;
        if (ip >= iend - 15) break;
      } while (sv == 255);
    }
    cpy = op + lit;
  safe_literal_copy:
    if (cpy > oend - 12 || ip + lit > iend - 8) {             // must be the last sequence
      if (ip + lit != iend || cpy > oend) return -1;
      out.lit(op, ip, lit);
      op += lit;
      break;
    }
    out.lit(op, ip, lit);
    ip += lit;
    op = cpy;
    off = (int64_t)(in.byte(ip) | in.byte(ip + 1) << 8);
    ip += 2;
    match = op - off;
    ml = token & 15;
  copy_match:
    if (ml == 15) {
      u32 sv;
      do {
        sv = in.byte(ip++);
        ml += sv;
        if (ip >= iend - 4) return -1;
      } while (sv == 255);
    }
    ml += 4;
  safe_match_copy:
    if (match < 0) return -1;
    cpy = op + ml;
    if (cpy > oend - 5) return -1;                            // the last 5 bytes are literals
    out.match(op, off, ml);
    op = cpy;
  }
  return op;
}

// The size prefix: the i32 LE size, or -1 where lz4::block::decompress returns Err before
// decoding (source < 4 bytes, negative size, size past LZ4_compressBound's limit).
__device__ __forceinline__ int64_t lz4_prefix(const uint8_t* s, u64 n) {
  if (n < 4) return -1;
  const int32_t v = (int32_t)((u32)s[0] | (u32)s[1] << 8 | (u32)s[2] << 16 | (u32)s[3] << 24);
  return (v < 0 || v > 0x7E000000) ? -1 : (int64_t)v;
}

// ------------------------------------------------------------------ HBM-to-HBM path
// Blocks past the LDS windows: the wave reads the compressed bytes and writes the output in
// global memory. A back-reference (a snappy copy, an LZ4 match) reads output bytes this wave
// stored earlier: their stores are drained first (s_waitcnt vmcnt(0)) and the reads are volatile
// (L2-served), so no stale L1 line can be returned.
__device__ __forceinline__ u32 out_byte(const uint8_t* p) {
  return *reinterpret_cast<const volatile uint8_t*>(p);
}
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// out[0 .. n) = in[0 .. n) by the wave (four bytes in flight per lane).
__device__ __forceinline__ void wave_copy_g(uint8_t* out, const uint8_t* in, u64 n) {
  u64 k = lane_id();
  for (; k + 192 < n; k += 256) {
    const uint8_t a = in[k], b = in[k + 64], c = in[k + 128], d = in[k + 192];
    out[k] = a;
    out[k + 64] = b;
    out[k + 128] = c;
    out[k + 192] = d;
  }
  for (; k < n; k += kWave) out[k] = in[k];
}

// out[d .. d + len) repeats the bytes `off` back (off <= d; 0 = zeros, the LZ4 offset-0 case):
// byte d + k is byte d - off + (k mod off).
__device__ __forceinline__ void match_copy_g(uint8_t* out, u64 d, u64 off, u64 len) {
  const u32 lane = lane_id();
  drain_stores();
  if (off == 0) {
    for (u64 k = lane; k < len; k += kWave) out[d + k] = 0;
    return;
  }
  for (u64 k0 = 0; k0 < len; k0 += kWave) {
    const u64 k = k0 + lane;
    u32 v = 0;
    if (k < len) v = out_byte(out + d - off + (k < off ? k : k % off));
    if (k < len) out[d + k] = (uint8_t)v;
  }
}

// snap's decompress_vec over global memory (the LDS path's checks, 64-bit lengths).
__device__ bool snappy_decode_global(const uint8_t* in, u64 n, u64 ip, uint8_t* out, u64 want) {
  u64 d = 0;
  while (ip < n) {
    u32 h[5];
#pragma unroll
    for (int q = 0; q < 5; q++) h[q] = ip + q < n ? uni(in[ip + q]) : 0u;
    const u32 tag = h[0], kind = tag & 3, t6 = tag >> 2;
    const u32 x = h[1] | h[2] << 8 | h[3] << 16 | h[4] << 24;
    u64 len, off = 0, hl;
    if (kind == 0) {
      const u32 nb = t6 >= 60 ? t6 - 59 : 0u;
      const u64 lx = nb == 0 ? t6 : (nb == 4 ? (u64)x : (u64)(x & ((1u << (8 * nb)) - 1)));
      len = lx + 1;
      hl = 1 + nb;
    } else {
      len = kind == 1 ? 4 + (t6 & 7) : t6 + 1;
      hl = kind == 1 ? 2 : (kind == 2 ? 3 : 5);
      off = kind == 1 ? (((tag >> 5) << 8) | (x & 0xFF)) : (kind == 2 ? (x & 0xFFFF) : x);
    }
    const u64 next = ip + hl + (kind == 0 ? len : 0);
    if (d + len > want || next > n || (kind != 0 && (off == 0 || off > d))) return false;
    if (kind == 0) wave_copy_g(out + d, in + ip + hl, len);
    else match_copy_g(out, d, off, len);
    ip = next;
    d += len;
  }
  return d == want;
}

struct Lz4GlobalUniSrc {         // wave-uniform, from global memory
  const uint8_t* p;
  __device__ u32 byte(int64_t i) const { return uni(p[i]); }
};
struct Lz4GlobalOut {            // wave-wide copies into global memory
  const uint8_t* in;
  uint8_t* out;
  __device__ void lit(int64_t op, int64_t ip, int64_t len) const {
    wave_copy_g(out + op, in + ip, (u64)len);
  }
  __device__ void match(int64_t op, int64_t off, int64_t len) const {
    match_copy_g(out, (u64)op, (u64)off, (u64)len);
  }
};

// The whole decode decision of a tag-3 block from global memory (per thread): its decoded
// length, or -1 (the codec's Err).
__device__ __forceinline__ int64_t lz4_block_length(const uint8_t* src, u64 src_bytes, u64 s, u64 len) {
  const int64_t size = lz4_prefix(src + s, len - 1);
  if (size < 0) return -1;
  return lz4_walk(Lz4LaneSrc{src, src_bytes, s + 4, s + 4 - (1ull << 62), 0}, (int64_t)len - 5, Lz4NoOut{}, size);
}

__device__ __forceinline__ int64_t lz4_block_length_lds(const uint8_t* src, u64 src_bytes, u64 s, u64 len,
                                                        uint8_t* win) {
  const int64_t size = lz4_prefix(src + s, len - 1);
  if (size < 0) return -1;
  return lz4_walk(Lz4LaneWinSrc{src, src_bytes, s + 4, s + 4 - (1ull << 62), win}, (int64_t)len - 5, Lz4NoOut{}, size);
}

__device__ __forceinline__ int64_t lz4_block_length_bytes(const uint8_t* blk, u64 len) {
  const int64_t size = lz4_prefix(blk, len - 1);
  if (size < 0) return -1;
  return lz4_walk(Lz4GlobalSrc{blk + 4}, (int64_t)len - 5, Lz4NoOut{}, size);
}

// ------------------------------------------------------------------ sizes
__global__ __launch_bounds__(256) void codec_sizes_kernel(CodecParams p) {
  __shared__ __attribute__((aligned(16))) uint8_t wins[256 * kLz4WinStride];
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n_blocks) return;
  const u64 s = p.ext[i], e = p.ext[i + 1], len = e - s;
  const u32 tag = len ? p.src[e - 1] : 0u;
  if (tag == 3) {
    if (p.claimed) {
      // the size prefix (lz4::block::decompress allocates that much, compress.rs:108-111): the
      // exact length of every stream the reference's compress wrote. A stream that decodes to
      // another length or fails sets the decompress's sticky word (tpz_decompress_check); a
      // claim no stream of this length can reach (LZ4 expands at most ~255x) takes the walk.
      const int64_t c = lz4_prefix(p.src + s, len - 1);
      if (c >= 0 && len > 5 && (u64)c <= 256 * (len - 5) + 64) {
        p.size[i] = (u64)c + 1;
        return;
      }
    }
    // the exact decoded length (LZ4 may decode fewer bytes than its prefix says); an Err
    // leaves a lone tag byte
    const int64_t r = p.src_bytes >= 16
        ? lz4_block_length_lds(p.src, p.src_bytes, s, len, wins + threadIdx.x * kLz4WinStride)
        : lz4_block_length_bytes(p.src + s, len);
    p.size[i] = r < 0 ? 1 : (u64)r + 1;
    return;
  }
  if (tag != 2) {                         // not compressed: copied unchanged
    p.size[i] = len;
    return;
  }
  u64 want = 0;
  const u32 h = snappy_header(p.src + s, len - 1, want);
  // an invalid preamble leaves an empty range (the decode reports it; the codec status says why)
  p.size[i] = h == 0 ? 0 : want + 1;
}

struct BlockMeta {
  u64 s, e, D0, D1;
  u32 tag;
};

// One LZ4 block (tag 3). Returns false when it does not fit the windows and this is not the
// last resort (the caller defers it); the last resort decodes past the windows from HBM.
template <u32 kIn, u32 kOut>
__device__ __forceinline__ bool lz4_block(const CodecParams& p, u32 b, const BlockMeta& m,
                                          uint8_t* in_win, uint8_t* out_win, bool last_resort) {
  const u32 lane = lane_id();
  const u64 s = m.s, len = m.e - m.s;
  uint8_t* dst = p.dst + m.D0;
  const u64 dn = m.D1 - m.D0;
  const bool fits = len - 1 + kInSlack <= kIn && dn + 16 <= kOut;
  if (!fits && !last_resort) return false;
  u32 st = TPZ_BLOCK_CODEC_ERROR;
  bool ok = false;
  const u32 a_out = (u32)(reinterpret_cast<uintptr_t>(dst) & 15);
  uint8_t* out = out_win + a_out;
  bool direct = false;          // the output went straight to dst
  if (dn < 2) {
    // an Err (the sizes pass gave it 1 byte) or an empty output: the decision again, from
    // global memory
    const int64_t r = p.src_bytes >= 16 ? lz4_block_length(p.src, p.src_bytes, s, len)
                                        : lz4_block_length_bytes(p.src + s, len);
    ok = r == 0 && dn == 1;
  } else if (!fits) {
    const int64_t size = lz4_prefix(p.src + s, len - 1);     // valid: dn >= 2
    const int64_t r = lz4_walk(Lz4GlobalUniSrc{p.src + s + 4}, (int64_t)len - 5,
                               Lz4GlobalOut{p.src + s + 4, dst}, size);
    ok = r >= 0 && (u64)r + 1 == dn;
    direct = true;
  } else {
    stage_aligned(p.src, p.src_bytes, s, (u32)(len - 1), in_win);
    __builtin_amdgcn_wave_barrier();
    const uint8_t* in = in_win + (u32)(s & 15);
    const int64_t size = lz4_prefix(p.src + s, len - 1);     // valid: dn >= 2
    const int64_t r = lz4_walk(Lz4LdsSrc{in + 4}, (int64_t)len - 5, Lz4WaveOut{in + 4, out}, size);
    __builtin_amdgcn_wave_barrier();
    ok = r >= 0 && (u64)r + 1 == dn;
  }
  if (ok && direct) {
    if (lane == 0) {
      dst[dn - 1] = 1;                                         // re-tagged Uncompress
      p.status[b] = TPZ_BLOCK_OK;
    }
  } else if (ok) {
    if (lane == 0) out[dn - 1] = 1;                            // re-tagged Uncompress
    __builtin_amdgcn_wave_barrier();
    store_aligned(out_win, dst, (u32)dn);
    if (lane == 0) p.status[b] = TPZ_BLOCK_OK;
  } else if (lane == 0) {
    if (dn) dst[dn - 1] = 0;                                   // decodes as BAD_TAG
    p.status[b] = (uint8_t)st;
    // a range of 2+ bytes for a stream that failed or decoded to another length: only claimed
    // sizes give one (the exact ones are 1 for an Err and the decoded length + 1 otherwise)
    if (dn >= 2 && p.inexact) atomicOr(p.inexact, 1u);
  }
  __builtin_amdgcn_wave_barrier();
  return true;
}

// One block. Returns false when it does not fit the windows (the caller defers it).
template <u32 kIn, u32 kOut>
__device__ __forceinline__ bool codec_block(const CodecParams& p, u32 b, const BlockMeta& m,
                                            uint8_t* in_win, uint8_t* out_win,
                                            bool last_resort STAMPS_ARG) {
  const u32 lane = lane_id();
  const u64 s = m.s, len = m.e - m.s;
  uint8_t* dst = p.dst + m.D0;
  const u64 dn = m.D1 - m.D0;
  if (len != 0 && m.tag == 3) return lz4_block<kIn, kOut>(p, b, m, in_win, out_win, last_resort);
  if (len == 0 || m.tag != 2) {                               // copied unchanged
    const u64 n = len < dn ? len : dn;
    for (u64 k = lane; k < n; k += kWave) dst[k] = p.src[s + k];
    if (lane == 0) p.status[b] = TPZ_BLOCK_OK;
    return true;
  }
  const bool fits = len - 1 + kInSlack <= kIn && dn + 16 <= kOut;
  u64 want = 0;
  u32 h = 0, st = TPZ_BLOCK_CODEC_ERROR;
  bool ok = false;
  const u32 a_in = (u32)(s & 15), a_out = (u32)(reinterpret_cast<uintptr_t>(dst) & 15);
  uint8_t* in = in_win + a_in;
  uint8_t* out = out_win + a_out;
  if (fits) {
    STAMP(5);
    stage_aligned(p.src, p.src_bytes, s, (u32)(len - 1), in_win);
    __builtin_amdgcn_wave_barrier();
    STAMP(1);
    // varint preamble from the staged bytes (at most 10, inside the block)
    const u32 v0 = lds_u32(in, 0), v1 = lds_u32(in, 4), v2 = lds_u32(in, 8);
    u64 v = 0;
    for (u32 i = 0; i < 10 && i < len - 1; i++) {
      const u32 c = ((i < 4 ? v0 : i < 8 ? v1 : v2) >> (8 * (i & 3))) & 0xFF;
      v |= (u64)(c & 0x7F) << (7 * i);
      if (!(c & 0x80)) {
        if (v <= 0xFFFFFFFFull) {
          want = v;
          h = i + 1;
        }
        break;
      }
    }
  } else {
    if (!last_resort) return false;
    // past the LDS windows: straight from HBM to HBM
    h = snappy_header(p.src + s, len - 1, want);
    const bool ok2 = h != 0 && want + 1 == dn &&
                     snappy_decode_global(p.src + s, len - 1, h, dst, want);
    if (lane == 0) {
      if (dn) dst[dn - 1] = ok2 ? 1 : 0;                       // re-tagged, or BAD_TAG
      p.status[b] = ok2 ? (uint8_t)TPZ_BLOCK_OK : (uint8_t)TPZ_BLOCK_CODEC_ERROR;
    }
    __builtin_amdgcn_wave_barrier();
    return true;
  }
  if (fits && h != 0 && want + 1 == dn) {
    STAMP(2);
    ok = snappy_decode(in, (u32)(len - 1), h, out, (u32)want STAMPS_PASS);
    __builtin_amdgcn_wave_barrier();
    STAMP(3);
  }
  if (ok) {
    if (lane == 0) out[want] = 1;                              // re-tagged Uncompress
    __builtin_amdgcn_wave_barrier();
    store_aligned(out_win, dst, (u32)(want + 1));
    if (lane == 0) p.status[b] = TPZ_BLOCK_OK;
    STAMP(4);
    SCOUNT(7, 1);
  } else {
    if (lane == 0) {
      if (dn) dst[dn - 1] = 0;                                 // decodes as BAD_TAG
      p.status[b] = (uint8_t)st;
    }
  }
  __builtin_amdgcn_wave_barrier();
  return true;
}

__device__ __forceinline__ u64 readlane64(u64 x, u32 k) {
  return ((u64)__builtin_amdgcn_readlane((u32)(x >> 32), k) << 32) |
         __builtin_amdgcn_readlane((u32)x, k);
}

// Each wave takes blocks wave0, wave0 + S, wave0 + 2S, ... (S = waves in the grid); their
// extents and tag bytes are loaded 64 blocks at a time, one block per lane.
__global__ __launch_bounds__(kWave * kSmallWaves) void codec_wave_kernel(CodecParams p) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kSmallWaves * (kGuard + kSmallIn + kSmallOut)];
  const u32 lane = lane_id();
  const u32 wid = uni(threadIdx.x >> 6);
  uint8_t* in_win = lds + wid * (kGuard + kSmallIn + kSmallOut) + kGuard;
  uint8_t* out_win = in_win + kSmallIn;
  const u32 S = gridDim.x * kSmallWaves;
#ifdef TPZ_CODEC_STAMPS
  Stamps st_;
#endif
  for (u32 g = blockIdx.x * kSmallWaves + wid; g < p.n_blocks; g += kWave * S) {
    const u32 bj = g + lane * S;
    const u32 bc = bj < p.n_blocks ? bj : p.n_blocks - 1;
    // after the lane kernels almost every block is final: one status load per 64 blocks, and
    // the metadata loads only where a block was left (the three dependent loads per group cost
    // 14 us over 2^18 blocks with nothing left)
    if (p.group_pass && !__ballot(p.status[bc] == kLeftForWaveKernel)) continue;
    BlockMeta mj;
    mj.s = p.ext[bc];
    mj.e = p.ext[bc + 1];
    mj.D0 = p.dst_ext[bc];
    mj.D1 = p.dst_ext[bc + 1];
    mj.tag = mj.e > mj.s ? p.src[mj.e - 1] : 0u;
    // blocks the group kernel decoded carry their final status; the rest are marked
    const u32 left = (!p.group_pass || p.status[bc] == kLeftForWaveKernel) ? 1u : 0u;
    const u32 cnt = uni((p.n_blocks - g + S - 1) / S < (u32)kWave ? (p.n_blocks - g + S - 1) / S
                                                                  : (u32)kWave);
    STAMP(0);
    for (u32 k = 0; k < cnt; k++) {
      if (!__builtin_amdgcn_readlane(left, k)) continue;
      BlockMeta m;
      m.s = readlane64(mj.s, k);
      m.e = readlane64(mj.e, k);
      m.D0 = readlane64(mj.D0, k);
      m.D1 = readlane64(mj.D1, k);
      m.tag = __builtin_amdgcn_readlane(mj.tag, k);
      const u32 b = g + k * S;
      if (!codec_block<kSmallIn, kSmallOut>(p, b, m, in_win, out_win, false STAMPS_PASS) &&
          lane == 0)
        p.defer_list[atomicAdd(p.defer_count, 1u)] = b;
      STAMP(5);
    }
  }
#ifdef TPZ_CODEC_STAMPS
  st_.flush(lane == 0);
#endif
}


// ------------------------------------------------------------------ snappy, one block per lane
// The wave-per-block element loop runs its ~70 wave-uniform instructions once per element per
// block. Here every lane walks its own block's element chain straight from HBM to HBM, so each
// header decode and copy instruction serves 64 blocks at once; the lanes diverge only in which
// copy path an element takes and for how many 16-byte pieces. The output is written in 16-byte
// pieces at the element's (unaligned) position: a piece that runs past the element holds bytes
// that later elements overwrite (the lane's stores land in program order), and no store passes the
// block's `want` bytes, so neighbouring blocks are never touched. Back-references read the lane's
// own earlier output (single-thread read-after-write through memory).
// Stores whose piece does not belong to the block go here instead (never read).
__device__ u128 g_store_sink[1024];
__device__ __forceinline__ uint8_t* sink_for_lane() {
  return reinterpret_cast<uint8_t*>(&g_store_sink[threadIdx.x & 1023]);
}

// The last bytes of a block: out[k .. room) = the low bytes of v, exact width (no byte past it)
__device__ __noinline__ void put_tail(uint8_t* o, u64 k, u128 v, u64 room) {
  const u32 r = (u32)(room - k);
  uint8_t* q = o + k;
  if (r & 8) { const u64 w = (u64)v; __builtin_memcpy(q, &w, 8); q += 8; v >>= 64; }
  if (r & 4) { const u32 w = (u32)v; __builtin_memcpy(q, &w, 4); q += 4; v >>= 32; }
  if (r & 2) { const uint16_t w = (uint16_t)v; __builtin_memcpy(q, &w, 2); q += 2; v >>= 16; }
  if (r & 1) *q = (uint8_t)v;
}

// Up to four pieces k0 + 16 j (j < 4, k0 + 16 j < len) of an element at o: whole pieces inside
// the block's room are stored (bytes past the element are rewritten by later elements), a piece
// past the room goes to the sink and its in-room bytes are stored exactly afterwards.
__device__ __forceinline__ void put4(uint8_t* o, u64 k0, const u128 (&v)[4], u64 len, u64 room) {
  uint8_t* sink = sink_for_lane();
  bool tail = false;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const u64 k = k0 + 16 * j;
    const bool whole = k + 16 <= room;
    tail |= !whole && k < len;
    st16u(whole ? o + k : sink, v[j]);
  }
  if (tail) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const u64 k = k0 + 16 * j;
      if (k + 16 > room && k < len) put_tail(o, k, v[j], room);
    }
  }
}

// The 16 bytes p[(r + i) mod off], i < 16, of the sequence with period off (< 16) whose first
// off bytes are pat's low bytes: the period rotated by r, then doubled in registers.
__device__ __forceinline__ u128 periodic16(u128 pat, u32 off, u32 r) {
  const u128 lo = pat >> (8 * r), hi = pat & (((u128)1 << (8 * r)) - 1);
  u128 v = (lo & (((u128)1 << (8 * (off - r))) - 1)) | (hi << (8 * (off - r)));
  for (u32 L = off; L < 16; L *= 2) v |= v << (8 * L);
  return v;
}

// A lane's element copies. The pieces of a copy are loaded together and then stored together,
// branch-free: a lane's loads and stores complete in order (one vmcnt), so any load issued after a
// store also waits for it; grouping keeps that to about one wait per element instead of one per
// piece. `pos` is the absolute output position in dst, `room` the block's bytes from there.
// out[pos .. pos + len) = src[q .. q + len)
__device__ __forceinline__ void lane_lit(const uint8_t* src, u64 src_bytes, u64 q, uint8_t* dst,
                                         u64 pos, u64 len, u64 room) {
  u128 v[4];
  for (u64 k = 0; k < len; k += 64) {
#pragma unroll
    for (int j = 0; j < 4; j++) v[j] = ld16c(src, src_bytes, q + k + 16 * j);
    put4(dst + pos, k, v, len, room);
  }
}

// out[pos .. pos + len) repeats the bytes `off` back (0 = zeros, LZ4's offset-0 match)
__device__ __forceinline__ void lane_match(uint8_t* dst, u64 dst_bytes, u64 pos, u64 off, u64 len,
                                           u64 room) {
  u128 v[4];
  uint8_t* o = dst + pos;
  if (off == 0 || off >= len || off >= 64) {
    // the source of every 64-byte round ends before it: final bytes (earlier rounds included)
    for (u64 k = 0; k < len; k += 64) {
#pragma unroll
      for (int j = 0; j < 4; j++)
        v[j] = off == 0 ? (u128)0
                        : ld16c(dst, dst_bytes, pos - off + k + (k + 16 * j < len ? 16 * j : 0));
      put4(o, k, v, len, room);
    }
  } else if (off < 16) {
    // period off: every piece from the off bytes before pos, in registers
    const u64 a = pos >= 16 ? pos - 16 : 0;
    const u128 w = ld16u(dst + a);
    const u128 pat = w >> (8 * (pos - a - off));
    const u32 o32 = (u32)off, s16 = 16u % o32;
    u32 r = 0;
    for (u64 k = 0; k < len; k += 64) {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        v[j] = periodic16(pat, o32, r);
        r += s16;
        r = r >= o32 ? r - o32 : r;
      }
      put4(o, k, v, len, room);
    }
  } else {
    // 16 <= off < len, off < 64: piece k reads piece k - off of this copy
    for (u64 k = 0; k < len; k += 16) {
      const u128 t = ld16u(o + k - off);
      if (k + 16 <= room) st16u(o + k, t);
      else put_tail(o, k, t, room);
    }
  }
}

#ifdef TPZ_CODEC_STAMPS
// lane kernel diagnostics: [0] wave cycles, [1] waves, [2] elements (all lanes), [3] wave loop
// trips, [4] literal rounds, [5] match rounds
__device__ unsigned long long g_lstamps[8];
#define LCOUNT(v) (v)++
#else
#define LCOUNT(v) (void)0
#endif

__device__ bool snappy_lane(const uint8_t* src, u64 src_bytes, u64 s, u64 n, u64 ip,
                            uint8_t* dst, u64 dst_bytes, u64 D0, u64 want, u32& elems) {
  u64 d = 0;
  u128 hv = ld16c(src, src_bytes, s + ip);
  while (ip < n) {
    // the tag and the 4 bytes after it (bytes past the block are don't-care: the checks below
    // reject any element that needs them)
    const u64 h = (u64)hv;
    const u32 tag = (u32)h & 0xFF, kind = tag & 3, t6 = tag >> 2;
    const u32 x = (u32)(h >> 8);
    u64 len, off = 0, hl;
    if (kind == 0) {
      const u32 nb = t6 >= 60 ? t6 - 59 : 0u;
      len = (u64)(nb == 0 ? t6 : (nb == 4 ? x : x & ((1u << (8 * nb)) - 1))) + 1;
      hl = 1 + nb;
    } else {
      len = kind == 1 ? 4 + (t6 & 7) : t6 + 1;
      hl = kind == 1 ? 2 : (kind == 2 ? 3 : 5);
      off = kind == 1 ? (((tag >> 5) << 8) | (x & 0xFF)) : (kind == 2 ? (x & 0xFFFF) : x);
    }
    const u64 next = ip + hl + (kind == 0 ? len : 0);
    // snap's Err: output overrun, element past the input, copy offset 0 or before the output
    if (d + len > want || next > n || (kind != 0 && (off == 0 || off > d))) return false;
    hv = ld16c(src, src_bytes, s + next);                    // the next header, in flight now
    LCOUNT(elems);
    if (kind == 0) lane_lit(src, src_bytes, s + ip + hl, dst, D0 + d, len, want - d);
    else lane_match(dst, dst_bytes, D0 + d, off, len, want - d);
    ip = next;
    d += len;
  }
  return d == want;
}

// LZ4 through lz4_walk, one block per lane: input bytes from a 16-byte register window that is
// reloaded when the walk leaves it; copies as above.
struct Lz4LaneOut {
  const uint8_t* src;
  u64 src_bytes, ibase;         // in[0] is src[ibase]
  uint8_t* dst;
  u64 dst_bytes, D0, r;         // the block's output: dst[D0 .. D0 + r)
  __device__ void lit(int64_t op, int64_t ip, int64_t len) const {
    lane_lit(src, src_bytes, ibase + (u64)ip, dst, D0 + (u64)op, (u64)len, r - (u64)op);
  }
  __device__ void match(int64_t op, int64_t off, int64_t len) const {
    lane_match(dst, dst_bytes, D0 + (u64)op, (u64)off, (u64)len, r - (u64)op);
  }
};

__device__ __forceinline__ void codec_lane_block(const CodecParams& p, u32 b, u32& elems);

// One thread per block. Takes the snappy and LZ4 blocks whose decoded length agrees with the sizes
// pass; every other block, and any block whose stream turns out invalid, gets status 0xFF and is
// left to codec_wave_kernel (which runs next, skips the rest and reports the codec's Err exactly).
__global__ __launch_bounds__(256) void codec_lane_kernel(CodecParams p) {
  const u32 b = blockIdx.x * 256 + threadIdx.x;
  u32 elems = 0;
#if defined(TPZ_CODEC_STAMPS) && defined(TPZ_CODEC_LANE_SNAPPY)
  const u64 t0 = __builtin_amdgcn_s_memtime();
  codec_lane_block(p, b, elems);
  const u64 t1 = __builtin_amdgcn_s_memtime();
  u32 mx = 0;
  for (int l = 0; l < 64; l++) mx = max(mx, (u32)__builtin_amdgcn_readlane(elems, l));
  atomicAdd(&g_lstamps[2], (unsigned long long)elems);
  if (lane_id() == 0) {
    atomicAdd(&g_lstamps[0], (unsigned long long)(t1 - t0));
    atomicAdd(&g_lstamps[1], 1ull);
    atomicAdd(&g_lstamps[3], (unsigned long long)mx);
  }
#else
  codec_lane_block(p, b, elems);
#endif
}

__device__ __forceinline__ void codec_lane_block(const CodecParams& p, u32 b, u32& elems) {
  if (b >= p.n_blocks) return;
  if (p.status[b] != kLeftForWaveKernel) return;              // decoded by a ring kernel
  const u64 s = p.ext[b], e = p.ext[b + 1], len = e - s;
  const u64 D0 = p.dst_ext[b], dn = p.dst_ext[b + 1] - D0;
  const u32 tag = len ? p.src[e - 1] : 0u;
  const u64 dst_bytes = p.dst_ext[p.n_blocks];
  // (tiny batches, errors, empty outputs and other tags: the wave kernel)
  bool ok = len > 1 && tag == 3 && dn >= 2 && p.src_bytes >= 16 && dst_bytes >= 16;
  if (!ok) return;                                            // status stays 0xFF
  if (ok && tag == 2) {
    u64 want = 0;
    const u32 h = snappy_header(p.src + s, len - 1, want);
    ok = h != 0 && want + 1 == dn &&
         snappy_lane(p.src, p.src_bytes, s, len - 1, h, p.dst, dst_bytes, D0, want, elems);
  } else if (ok) {
    const int64_t size = lz4_prefix(p.src + s, len - 1);
    ok = size >= 0;
    if (ok) {
      Lz4LaneSrc in{p.src, p.src_bytes, s + 4, s + 4 - (1ull << 62), 0};
      const int64_t r = lz4_walk(in, (int64_t)len - 5,
                                 Lz4LaneOut{p.src, p.src_bytes, s + 4, p.dst, dst_bytes, D0, dn - 1},
                                 size);
      ok = r >= 0 && (u64)r + 1 == dn;
    }
  }
  if (ok) p.dst[D0 + dn - 1] = 1;                              // re-tagged Uncompress
  p.status[b] = ok ? (uint8_t)TPZ_BLOCK_OK : kLeftForWaveKernel;
}

// ------------------------------------------------------------------ snappy, one block per lane, LDS ring
// Per-lane 16-byte stores to 64 different blocks run at ~1 TB/s on this chip, while a wave whose
// lanes cover whole lines in groups (4 lanes per 64-byte line) stores at 3.6-4.8 TB/s
// (tools/ubench_lane.hip). So each lane decodes its block into a 256-byte ring in LDS (4 lines of
// 64 bytes at the output's absolute alignment) and, after every step, the wave stores the lines
// its lanes completed cooperatively: 16 lines per store instruction. The line a block shares with
// its neighbour at either end is stored by its own lane with exact-width stores.
// The ring is written in aligned 16-byte slots only: a step's bytes are funnelled into slots in
// registers (the slot holding the output frontier is kept in a register too, so no slot is read
// back before it is rewritten); unaligned reads are two aligned slot reads and a funnel. So no
// write passes the frontier's slot, and two lines (128 bytes per lane, 16 waves per CU) hold
// the current line and the previous one intact at every step.
// A step produces at most 64 bytes of one element per lane. Copy sources come from the ring when
// they lie in the current or the previous line, otherwise from the lines already stored: those
// loads wait for the wave's earlier stores (vmcnt); the stores came from this wave, so this CU's
// L1 holds no stale copy. A step issues one set of four 16-byte loads for every lane: a literal's
// source bytes or a far copy's stored lines (one set instead of one per descriptor: 1.351 ->
// 1.314 ms per 2^18 4kc blocks).
constexpr u32 kRingWG = 256;                                 // blocks (threads) per workgroup
constexpr u32 kRing = 128;                                   // 4 workgroups (16 waves) per CU
constexpr u32 kRingLine = 64, kRingStep = 64;
// 16-byte pieces a step can take. A literal's steps are 64 bytes, but its final step may take up
// to 16 kPieces bytes as long as it ends by Pl + 128 (every line it completes is then still
// intact in the ring when the step's stores read it): a 65-80 byte literal is one step instead
// of two. (Per 2^18 4kc blocks: 4 pieces 1.22 ms, 5 pieces 1.15 ms, steps of up to two whole
// lines with 8 pieces 1.22-1.24 ms; profiles/r2/codec_ring.jsonl.)
#ifndef TPZ_CODEC_PIECES
#define TPZ_CODEC_PIECES 5
#endif
constexpr u32 kPieces = TPZ_CODEC_PIECES;
static_assert(kPieces >= 4 && kPieces <= 7, "a step ends by Pl + 128");
// bytes a literal step starting at P takes of the `rem` left
__device__ __forceinline__ u32 lit_step(u32 P, u32 rem) {
  const u32 lim = min(16 * kPieces, 128u - (P & 63u));
  return rem <= lim ? rem : kRingStep;
}
// the length of the final step of a literal of len bytes whose first step starts at P (steps of
// 64 keep P mod 64, and with it the limit, the same)
__device__ __forceinline__ u32 lit_final(u32 P, u32 len) {
  const u32 lim = min(16 * kPieces, 128u - (P & 63u));
  return len <= lim ? len : len - 64 * ((len - lim + 63) / 64);
}
static_assert(kRingWG * kRing + (kRingWG / kWave) * kWave * 12 <= (kRing == 128 ? 40960 : 81920),
              "ring LDS");

__device__ __forceinline__ u128 lds16(const uint8_t* q) {
  return *reinterpret_cast<const u128*>(q);                  // aligned
}
__device__ __forceinline__ void lds16w(uint8_t* q, u128 v) { *reinterpret_cast<u128*>(q) = v; }
__device__ __forceinline__ u128 lowbytes(u128 v, u32 m) {    // the low m (< 16) bytes of v
  return v & (((u128)1 << (8 * m)) - 1);
}

// The 16 ring bytes at absolute address a (R[a % kRing ..], any alignment).
__device__ __forceinline__ u128 ring_read(const uint8_t* R, u32 a) {
  const u32 o = a & (kRing - 1), m = o & 15, o0 = o & ~15u;
  const u128 s0 = lds16(R + o0), s1 = lds16(R + ((o0 + 16) & (kRing - 1)));
  return m ? (s0 >> (8 * m)) | (s1 << (8 * (16 - m))) : s0;
}

// Writes the step's output bytes [P, P + c) (c <= 16 kPieces; v[j] = bytes [P + 16 j, P + 16 j +
// 16)) into the ring's aligned slots. acc holds the slot containing P (its bytes below P are the
// output); on return it holds the slot containing P + c.
__device__ __forceinline__ void ring_emit(uint8_t* R, u32 P, u32 c, const u128 (&v)[kPieces], u128& acc) {
  const u32 m = P & 15, K = (m + c + 15) >> 4, Kn = (m + c) >> 4;
  const u32 A = P & ~15u;
  // the new frontier's slot keeps its upper half when the frontier is in its lower half: the
  // ring then holds [roundup8(P) - kRing, P) intact (a copy 120 bytes back always from LDS)
  const bool half = ((P + c) & 15u) != 0 && ((P + c) & 15u) <= 8;
  u128 carry = m ? lowbytes(acc, m) : (u128)0, nacc = acc;
#pragma unroll
  for (int k = 0; k <= (int)kPieces; k++) {
    const u128 cur = k < (int)kPieces ? v[k < (int)kPieces ? k : 0] : (u128)0;
    const u128 slot = m ? carry | (cur << (8 * m)) : cur;
    if ((u32)k < K) {
      uint8_t* q = R + ((A + 16 * k) & (kRing - 1));
      if ((u32)k == Kn && half) *reinterpret_cast<u64*>(q) = (u64)slot;
      else lds16w(q, slot);
    }
    if ((u32)k == Kn) nacc = slot;
    carry = m ? cur >> (8 * (16 - m)) : (u128)0;
  }
  acc = nacc;
}

// dst[x0 .. x1) from the ring, exact width (the lines a block shares with its neighbours)
__device__ __forceinline__ void ring_store_exact(const uint8_t* R, uint8_t* dst, u32 x0, u32 x1) {
  for (u32 k = 0; x0 + k < x1; k += 16) {
    const u128 v = ring_read(R, x0 + k);
    if (x0 + k + 16 <= x1) st16u(dst + x0 + k, v);
    else put_tail(dst + x0, k, v, x1 - x0);
  }
}

// The ring body for snappy (kCodec 2) and LZ4 (kCodec 3) blocks: they differ only in how an
// element is decoded (an LZ4 sequence is a literal element, then a copy element).
template <int kCodec>
__device__ __forceinline__ void ring_body(CodecParams p) {
  __shared__ __attribute__((aligned(16))) uint8_t rings[kRingWG * kRing];
  __shared__ u32 fl_addr[kRingWG / kWave][kWave];
  __shared__ u32 fl_lane[kRingWG / kWave][kWave];
  const u32 lane = lane_id(), wid = threadIdx.x >> 6;
  uint8_t* R = rings + threadIdx.x * kRing;
  const u32 b = blockIdx.x * kRingWG + threadIdx.x;
  const u64 dst_bytes = p.dst_ext[p.n_blocks];
  // a buffer descriptor over the whole source for the header loads (batches below 2 GiB)
  const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.src, (short)0, (int)(p.src_bytes < 0x7FFFFFF0ull ? p.src_bytes : 0x7FFFFFF0ull),
      0x00020000);

  // Every position is a 32-bit offset: live blocks need src_bytes and dst_bytes below 2^31.
  bool live = false;
  u32 s = 0, n = 0, ip = 0, want = 0, D0 = 0, dn = 0;
  // LZ4: liblz4's output limit (the size prefix) and where its walk stands: bit 0 = the safe
  // loop (entered for good once a sequence leaves the fast loop, or from the start when the
  // limit is below 64), bit 1 = the current sequence took the safe loop's two-stage shortcut
  u32 oend = 0, lzm = 0;
  // (LZ4: the snappy pass marked every block it did not decode; the status first, so that a
  // batch without LZ4 blocks costs this pass one load per lane)
  if (b < p.n_blocks && (kCodec != 3 || p.status[b] == kLeftForWaveKernel)) {
#ifdef TPZ_CODEC_ONCHIP
    const u32 bx = b & 4095u;   // timing build: the same 4096 blocks again and again (on chip)
#else
    const u32 bx = b;
#endif
    const u64 s64 = p.ext[bx], e64 = p.ext[bx + 1], len = e64 - s64;
    const u64 D064 = p.dst_ext[bx], dn64 = p.dst_ext[bx + 1] - D064;
    const u32 tag = len ? p.src[e64 - 1] : 0u;
    live = len > 1 && tag == (u32)kCodec && dn64 >= 2 && p.src_bytes >= 16 && dst_bytes >= 16 &&
           dst_bytes < 0x7FFFFFF0ull && p.src_bytes < 0x7FFFFFF0ull;
    if (live) {
      u64 want64 = 0;
      u32 h = 0;
      if constexpr (kCodec == 2) {
        h = snappy_header(p.src + s64, len - 1, want64);
        live = h != 0 && want64 + 1 == dn64;
      } else {
        // u32 LE size prefix, then the block stream (compress.rs:108-111). dn - 1 is either the
        // exact decoded length (tpz_decompressed_sizes ran liblz4's walk) or the size prefix
        // itself (tpz_decompressed_sizes_claimed: no walk ran). So this pass applies liblz4's
        // acceptance rules itself, sequence by sequence, with the walk's own output limit (the
        // prefix: lz4_walk's oend); a block whose stream breaks one, or that this pass finds
        // anything unusual in, is left to the lane kernel, which runs lz4_walk.
        want64 = dn64 - 1;
        h = 4;
        const int64_t pre = lz4_prefix(p.src + s64, len - 1);
        live = pre >= 0 && len - 1 > 4 && pre < 0x7FFFFFF0;
        oend = live ? (u32)pre : 0u;
        lzm = oend >= 64 ? 0u : 1u;
      }
      s = (u32)s64;
      ip = h;
      n = (u32)(len - 1);
      want = (u32)want64;
      D0 = (u32)D064;
      dn = (u32)dn64;
    }
    if constexpr (kCodec == 2) {
      if (!live) p.status[b] = kLeftForWaveKernel;
    }
  }
  const u32 src_bytes = live ? (u32)p.src_bytes : 0u;
  u32 d = 0;                                  // bytes produced
  const u32 head_end = (D0 + kRingLine - 1) & ~(kRingLine - 1);
  u32 fl = D0;                                // bytes below fl are stored
  u128 hv = live ? ld16c(p.src, p.src_bytes, s + ip) : (u128)0;
  u32 hvv = 16;                               // hv holds the input bytes [ip, ip + hvv)
  u128 acc = 0;                               // the ring slot holding the frontier D0 + d
  u32 ek = 0;                                 // element: 0 literal, 1 copy
  u32 erem = 0, esrc = 0, eoff = 0;
  bool need_off = false;                      // LZ4: the next header is a match's offset part
  u32 mln = 0;                                // LZ4: the match-length nibble of the token
#ifdef TPZ_CODEC_STAMPS
  const u64 t0 = __builtin_amdgcn_s_memtime();
  u64 trips = 0, gtrips = 0, elems = 0;
#endif

  // Every block of the batch is in flight at once, one per lane, so no wave can take over the
  // blocks of a slower one: the kernel lasts as long as its slowest waves. The issue arbiter
  // favours the oldest wave, so the waves of a CU do not progress at one speed (the decode's wave
  // path: the first four finished 0.58 ms before the last four). The wave's priority rotates
  // every trip instead (offset per wave): snappy 1.19/1.15 -> 1.14/1.12 ms, LZ4 1.23 -> 1.19 ms
  // per 2^18 4kc blocks (profiles/r3/wave_chunks.jsonl).
  u32 rot = blockIdx.x * 4u + (threadIdx.x >> 6);
  while (__ballot(live)) {
    switch (uni(rot++) & 3u) {
      case 0: __builtin_amdgcn_s_setprio(0); break;
      case 1: __builtin_amdgcn_s_setprio(1); break;
      case 2: __builtin_amdgcn_s_setprio(2); break;
      default: __builtin_amdgcn_s_setprio(3); break;
    }
#ifdef TPZ_CODEC_STAMPS
    trips++;
#endif
    bool finish = false, fail = false;
    if (live && erem == 0) {
      if (ip >= n) {
        finish = true;
      } else if constexpr (kCodec == 3) {
        // LZ4 sequence (lz4 block format): token = literal length (high nibble) | match length
        // - 4 (low nibble); 15 continues with bytes until one is not 255; literals; u16 LE
        // offset; match-length continuation bytes. Decoded from the 16 header bytes in hv.
        auto hb = [&](u32 i) -> u32 { return (u32)(hv >> (8 * i)) & 0xFFu; };
        u32 o = 0, len = 0, off = 0;
        bool bad = false, is_lit = false;
        // liblz4 1.9.3's acceptance (lz4_walk, oracle/tpz_lz4.c:53-173), in positions relative to
        // the block (the stream's iend is n, its oend the prefix): rej = the walk returns Err
        const int I = (int)n, O = (int)oend, op = (int)d;
        bool rej = false;
        if (!need_off) {
          const u32 t = hb(0);
          u32 lit = t >> 4;
          mln = t & 15u;
          o = 1;
          if (lit == 15) {
            u32 x;
            do {
              bad = bad || o >= hvv;
              x = bad ? 0u : hb(o);
              lit += x;
              o++;
            } while (x == 255 && !bad);
          }
          // the literal part. (Where the walk stops reading a length early, 15 bytes before the
          // input end, its literal ends at the input end and this parse's runs past it: next > n.)
          const int ipt = (int)ip, ipL = ipt + (int)o, L = (int)lit;
          const bool l15 = (t >> 4) == 15;
          bool sl = false;                    // goes to safe_literal_copy
          if (!(lzm & 1u)) {                  // the fast loop
            if (l15) {
              rej = ipt + 1 >= I - 15;
              sl = op + L > O - 32 || ipL + L > I - 32;
            } else {
              sl = ipt + 1 > I - 17;
            }
          } else if (!l15 && ipt + 1 < I - 16 && op <= O - 32) {
            lzm |= 2u;                        // the two-stage shortcut: no end checks here
          } else {
            rej = l15 && ipt + 1 >= I - 15;
            sl = true;
          }
          if (sl) {
            lzm |= 1u;
            // near either end the sequence must be the last: it consumes the input exactly
            if (op + L > O - 12 || ipL + L > I - 8) rej = rej || ipL + L != I || op + L > O;
          }
          if (lit) {
            is_lit = true;
            len = lit;
          }
        }
        if (!is_lit && !bad) {                // the offset part (right after the token when no
          bad = o + 2 > hvv;                  // literal precedes it)
          off = bad ? 0u : hb(o) | hb(o + 1) << 8;
          o += 2;
          u32 ml = mln;
          if (ml == 15 && !bad) {
            u32 x;
            do {
              bad = bad || o >= hvv;
              x = bad ? 0u : hb(o);
              ml += x;
              o++;
            } while (x == 255 && !bad);
          }
          len = ml + 4;
          // the match part: a length continuation must end 5 bytes before the input end, and a
          // match checked against the output end (the fast loop checks it from 64 bytes before,
          // the shortcut not at all) must leave the last 5 bytes to literals
          const int ipM = (int)ip + (int)o, M = (int)len;
          const bool m15 = mln == 15, late = m15 && ipM >= I - 4;
          if (!(lzm & 1u)) {
            rej = rej || late;
            if (op + M >= O - 64) {
              lzm |= 1u;
              rej = rej || op + M > O - 5;
            }
          } else if (!((lzm & 2u) && !m15 && off >= 8)) {
            rej = rej || late || op + M > O - 5;
          }
          lzm &= 1u;
        }
        const u32 next = ip + o + (is_lit ? len : 0u);
        if (bad || rej || d + len > want || next > n || next < ip ||
            (!is_lit && (off == 0 || off > d))) {
          fail = true;
        } else {
          ek = is_lit ? 0u : 1u;
          erem = len;
          esrc = s + ip + o;
          eoff = off;
          need_off = is_lit;
          ip = next;
          const u32 used = is_lit ? o + len : o;
          hv = used < hvv ? hv >> (8 * used) : (u128)0;
          hvv = used < hvv ? hvv - used : 0u;
          if (hvv < 8 && next < n) {          // the next header, in flight during the element
            hv = s + next + 16 <= src_bytes
                     ? __builtin_bit_cast(u128, __builtin_amdgcn_raw_buffer_load_b128(srs, s + next, 0, 0))
                     : ld16c(p.src, p.src_bytes, s + next);
            hvv = 16;
          }
#ifdef TPZ_CODEC_STAMPS
          elems++;
#endif
        }
      } else {
        const u32 h0 = (u32)hv, x = (u32)(hv >> 8);
        const u32 tag = h0 & 0xFF, kind = tag & 3, t6 = tag >> 2;
        u32 len, off = 0, hl;
        bool big = false;                     // a 4-byte literal length past any output
        if (kind == 0) {
          const u32 nb = t6 >= 60 ? t6 - 59 : 0u;
          const u32 l0 = nb == 0 ? t6 : (nb == 4 ? x : x & ((1u << (8 * nb)) - 1));
          big = l0 >= 0x7FFFFFF0u;
          len = l0 + 1;
          hl = 1 + nb;
        } else {
          len = kind == 1 ? 4 + (t6 & 7) : t6 + 1;
          hl = kind == 1 ? 2 : (kind == 2 ? 3 : 5);
          off = kind == 1 ? (((tag >> 5) << 8) | (x & 0xFF)) : (kind == 2 ? (x & 0xFFFF) : x);
        }
        const u32 next = ip + hl + (kind == 0 ? len : 0);
        // snap's Err: output overrun, element past the input, copy offset 0 or before the output
        if (big || d + len > want || next > n || next < ip ||
            (kind != 0 && (off == 0 || off > d))) {
          fail = true;
        } else {
          ek = kind == 0 ? 0u : 1u;
          erem = len;
          esrc = s + ip + hl;
          eoff = off;
          ip = next;
          // the next header: still in hv after a copy or a short literal (a header is at most 5
          // bytes), else loaded now, in flight while this element is produced (clamped near the
          // end of the source)
          const u32 used = kind == 0 ? (hl + len < 16 ? hl + len : 16) : hl;
          hv = used < 16 ? hv >> (8 * used) : (u128)0;
          hvv = hvv > used ? hvv - used : 0u;
          // a literal whose final step's last piece ends 5..15 bytes past the literal carries the
          // next header: taken from that piece when the literal completes (hvv = 0 until then)
          const u32 rf = kind == 0 ? lit_final(D0 + d, len) & 15 : 0u;
          const bool from_lit = kind == 0 && hvv < 5 && rf >= 1 && rf <= 11 &&
                                s + next + 5 <= src_bytes;
          if (from_lit) hvv = 0;
          else if (hvv < 5) {
            hv = s + next + 16 <= src_bytes
                     ? __builtin_bit_cast(u128, __builtin_amdgcn_raw_buffer_load_b128(srs, s + next, 0, 0))
                     : ld16c(p.src, p.src_bytes, s + next);
            hvv = 16;
          }
#ifdef TPZ_CODEC_STAMPS
          elems++;
#endif
        }
      }
    }
    // produce up to kRingStep bytes of the current element (a copy with off >= 16: at most off,
    // so every source byte precedes the step)
    const bool prod = live && !finish && !fail && erem > 0;
    const u32 P = D0 + d;
    const bool lit = ek == 0, far = !lit && eoff >= 16;
    u32 c = !prod ? 0u : lit ? lit_step(P, erem) : (erem < kRingStep ? erem : kRingStep);
    if (prod && far && eoff < c) c = eoff;
    const u32 Pl = P & ~(kRingLine - 1);
    // The ring holds [roundup8(P) - kRing, P) intact: no write passes the frontier's 8-byte
    // half-slot, so the bytes past it still hold the bytes kRing before (a far copy of an
    // entry 120 bytes back is served from the ring; with whole 16-byte slots only about half
    // of them were). Everything below Pl is stored (the lines completed before this step).
    const u32 Pr = (P + 7) & ~7u;
    const u32 ring_lo = Pr >= kRing ? Pr - kRing : 0u;
    const u32 q0 = P - eoff;                                          // a copy's first source byte
    const bool gcopy = prod && far && q0 < ring_lo;
    // the 16-byte pieces this step loads from memory (a prefix of the step's four): a literal's,
    // or a far copy's pieces that start below the ring (the others come from the ring)
    const bool tail = lit && esrc + 16 * kPieces + 16 > src_bytes;
    const u32 cp = (c + 15) >> 4;
    const u32 np = !prod ? 0u : lit ? (tail ? 0u : cp)
                 : !gcopy ? 0u : min(cp, (ring_lo - q0 + 15) >> 4);
    if (__ballot(gcopy)) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stored lines landed
#ifdef TPZ_CODEC_STAMPS
      gtrips++;
#endif
    }
    if (prod) {
      // One set of four 16-byte global loads serves every lane: a literal's source bytes, or the
      // stored lines a far copy reads (the wave's own stores: same CU, visible after the vmcnt
      // wait above). Pieces a lane does not need are exec-masked off.
      u128 v[kPieces];
      const uint8_t* base = lit ? p.src + esrc : p.dst + q0;
#pragma unroll
      for (int j = 0; j < (int)kPieces; j++) v[j] = 0;
#pragma unroll
      for (int j = 0; j < (int)kPieces; j++)
        if ((u32)j < np) v[j] = *reinterpret_cast<const u128 __attribute__((aligned(1)))*>(base + 16 * j);
      if (lit) {
        if (tail)
#pragma unroll
          for (int j = 0; j < (int)kPieces; j++) v[j] = ld16c(p.src, p.src_bytes, esrc + 16 * j);
        esrc += c;
        if (kCodec == 2 && c == erem && hvv == 0) {
          const u32 r16 = c & 15, last = (c - 1) >> 4;
          u128 lp = v[0];
#pragma unroll
          for (int j = 1; j < (int)kPieces; j++) lp = last == (u32)j ? v[j] : lp;
          hv = lp >> (8 * r16);
          hvv = 16 - r16;
        }
      } else if (!far) {
        const u128 pat = ring_read(R, P - 16) >> (8 * (16 - eoff));
        const u32 s16 = 16u % eoff;
        u32 r = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
          v[j] = periodic16(pat, eoff, r);
          r += s16;
          r = r >= eoff ? r - eoff : r;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; j++)
          if ((u32)j >= np && (u32)j < cp) v[j] = ring_read(R, q0 + 16 * j);
      }
      ring_emit(R, P, c, v, acc);
      d += c;
      erem -= c;
    }
    if (fail) {
      live = false;
      p.status[b] = kLeftForWaveKernel;
    }
    if (finish) {
      live = false;
      // (LZ4: liblz4's walk ends only after a sequence's literals; after a match it reads a
      // token past the input and fails)
      if (d == want && (kCodec != 3 || need_off)) {
        // re-tagged Uncompress: the tag byte joins the frontier slot
        const u32 T = D0 + want;
        const u32 m = T & 15;
        const u128 slot = lowbytes(acc, m) | ((u128)1 << (8 * m));
        lds16w(R + ((T & ~15u) & (kRing - 1)), slot);
        ring_store_exact(R, p.dst, fl, D0 + dn);
        fl = D0 + dn;
        p.status[b] = TPZ_BLOCK_OK;
      } else {
        p.status[b] = kLeftForWaveKernel;
      }
    }
    // the head line (shared with the previous block) once complete, then whole lines
    const u32 F = D0 + d;
    if (live && fl < head_end && F >= head_end) {
      ring_store_exact(R, p.dst, fl, head_end);
      fl = head_end;
    }
    for (;;) {
      const bool has = live && fl >= head_end && fl + kRingLine <= F;
      const u64 mk = __ballot(has);
      if (mk == 0) break;
      const u32 cnt = __builtin_popcountll(mk);
      if (has) {
        const u32 k = __builtin_amdgcn_mbcnt_hi((u32)(mk >> 32), __builtin_amdgcn_mbcnt_lo((u32)mk, 0u));
        fl_addr[wid][k] = fl;
        fl_lane[wid][k] = lane;
      }
      // LDS written and read back by this wave only: the LDS runs one wave's instructions in
      // order, so a compiler barrier suffices (a wavefront fence also waits for every
      // outstanding global load and store, s_waitcnt vmcnt(0))
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
      for (u32 q = 0; q < cnt; q += kWave / 4) {
        const u32 k = q + (lane >> 2);
        if (k < cnt) {
          const u32 a = fl_addr[wid][k];
          const uint8_t* Rs = rings + (wid * kWave + fl_lane[wid][k]) * kRing;
          const u32 o = (a & (kRing - 1)) + 16 * (lane & 3);
          st16u(p.dst + a + 16 * (lane & 3), lds16(Rs + o));
        }
      }
      __builtin_amdgcn_wave_barrier();
      if (has) fl += kRingLine;
    }
  }
#ifdef TPZ_CODEC_STAMPS
  const u64 t1 = __builtin_amdgcn_s_memtime();
  atomicAdd(&g_lstamps[5], (unsigned long long)elems);
  if (lane == 0) {
    atomicAdd(&g_lstamps[0], (unsigned long long)(t1 - t0));
    atomicAdd(&g_lstamps[1], 1ull);
    atomicAdd(&g_lstamps[3], (unsigned long long)trips);
    atomicAdd(&g_lstamps[4], (unsigned long long)gtrips);
  }
#endif
}

// (the first kernel of the step zeroes the deferred-block counter the wave kernel appends to and
// the big kernel reads: a memset of 4 bytes was a 4 us fill kernel of its own)
__global__ __launch_bounds__(kRingWG) void snappy_ring_kernel(CodecParams p) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *p.defer_count = 0;
  ring_body<2>(p);
}
__global__ __launch_bounds__(kRingWG) void lz4_ring_kernel(CodecParams p) { ring_body<3>(p); }

__global__ __launch_bounds__(kWave) void codec_big_kernel(CodecParams p) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kGuard + kBigIn + kBigOut];
  const u32 cnt = uni(*p.defer_count);
  for (u32 it = blockIdx.x; it < cnt; it += gridDim.x) {
    const u32 b = uni(p.defer_list[it]);
    BlockMeta m;
    m.s = uni64(p.ext[b]);
    m.e = uni64(p.ext[b + 1]);
    m.D0 = uni64(p.dst_ext[b]);
    m.D1 = uni64(p.dst_ext[b + 1]);
    m.tag = m.e > m.s ? uni(p.src[m.e - 1]) : 0u;
#ifdef TPZ_CODEC_STAMPS
    Stamps st_;
#endif
    codec_block<kBigIn, kBigOut>(p, b, m, lds + kGuard, lds + kGuard + kBigIn, true STAMPS_PASS);
  }
}

}  // namespace

#ifdef TPZ_CODEC_STAMPS
extern "C" int tpz_debug_codec_stamps(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_cstamps), sizeof(g_cstamps)) != hipSuccess) return 1;
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_cstamps), z, sizeof(z)) != hipSuccess) return 1;
  }
  return 0;
}
#endif

#ifdef TPZ_CODEC_STAMPS
extern "C" int tpz_debug_lane_stamps(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lstamps), sizeof(g_lstamps)) != hipSuccess) return 1;
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_lstamps), z, sizeof(z)) != hipSuccess) return 1;
  }
  return 0;
}
#endif

void launch_codec_sizes(const CodecLaunch& a, hipStream_t stream) {
  CodecParams p{};
  p.src = a.src;
  p.ext = a.ext;
  p.src_bytes = a.src_bytes;
  p.n_blocks = a.n_blocks;
  p.size = a.size;
  p.claimed = a.claimed ? 1u : 0u;
  hipLaunchKernelGGL(codec_sizes_kernel, dim3((a.n_blocks + 255) / 256), dim3(256), 0, stream, p);
}

void launch_decompress(const CodecLaunch& a, hipStream_t stream) {
  CodecParams p{};
  p.src = a.src;
  p.ext = a.ext;
  p.src_bytes = a.src_bytes;
  p.n_blocks = a.n_blocks;
  p.dst = a.dst;
  p.dst_ext = a.dst_ext;
  p.status = a.status;
  p.defer_list = a.defer_list;
  p.defer_count = a.defer_count;
  p.inexact = a.inexact;
  if (a.n_blocks) {
    p.group_pass = 1;
    hipLaunchKernelGGL(snappy_ring_kernel, dim3((a.n_blocks + kRingWG - 1) / kRingWG), dim3(kRingWG),
                       0, stream, p);
    hipLaunchKernelGGL(lz4_ring_kernel, dim3((a.n_blocks + kRingWG - 1) / kRingWG), dim3(kRingWG),
                       0, stream, p);
    hipLaunchKernelGGL(codec_lane_kernel, dim3((a.n_blocks + 255) / 256), dim3(256), 0, stream, p);
  }
  u32 grid = (a.n_blocks + kSmallWaves - 1) / kSmallWaves;
  if (grid > a.num_cus) grid = a.num_cus;
  if (grid == 0) grid = 1;
  hipLaunchKernelGGL(codec_wave_kernel, dim3(grid), dim3(kWave * kSmallWaves), 0, stream, p);
  hipLaunchKernelGGL(codec_big_kernel, dim3(a.num_cus), dim3(kWave), 0, stream, p);
}

}  // namespace tpz
