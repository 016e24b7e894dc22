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
// 64 KiB input / 94 KiB output windows.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tpz_internal.h"

namespace tpz {

namespace {

typedef uint32_t u32;
typedef uint64_t u64;

constexpr int kWave = 64;
constexpr int kSmallWaves = 16;
constexpr u32 kSmallIn = 4608, kSmallOut = 5120;     // per-wave windows of the 16-wave kernel
constexpr u32 kBigIn = 65536, kBigOut = 94208;       // the one-wave kernel
constexpr u32 kInSlack = 16 + 8;                     // staging offset (< 16) + header overread
static_assert(kSmallWaves * (kSmallIn + kSmallOut) <= 163840, "small LDS");
static_assert(kBigIn + kBigOut <= 163840, "big LDS");

__device__ __forceinline__ u32 lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
__device__ __forceinline__ u32 uni(u32 x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ u64 uni64(u64 x) {
  const u32 lo = __builtin_amdgcn_readfirstlane((u32)x);
  const u32 hi = __builtin_amdgcn_readfirstlane((u32)(x >> 32));
  return ((u64)hi << 32) | lo;
}

// Little-endian u32 at any LDS byte offset (two aligned reads + alignbyte), wave-uniform.
__device__ __forceinline__ u32 lds_u32(const uint8_t* base, u32 a) {
  const u32* p = reinterpret_cast<const u32*>(base + (a & ~3u));
  return uni(__builtin_amdgcn_alignbyte(p[1], p[0], a & 3u));
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
};

// ------------------------------------------------------------------ sizes
__global__ __launch_bounds__(256) void codec_sizes_kernel(CodecParams p) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n_blocks) return;
  const u64 s = p.ext[i], e = p.ext[i + 1], len = e - s;
  if (len == 0 || p.src[e - 1] != 2) {   // not snappy: copied unchanged
    p.size[i] = len;
    return;
  }
  u64 want = 0;
  const u32 h = snappy_header(p.src + s, len - 1, want);
  // an invalid preamble leaves an empty range; a declared length no device decode could take
  // leaves a lone tag byte (the decode reports it; the codec status says why)
  p.size[i] = h == 0 ? 0 : (want + 1 <= TPZ_MAX_BLOCK_BYTES ? want + 1 : 1);
}

// ------------------------------------------------------------------ per-block work
// Copies LDS bytes [lo, lo + n) of `win` to global [g, g + n): 16-byte stores for the aligned
// pieces strictly inside, byte stores for the (shared) edge pieces.
__device__ __forceinline__ void store_bytes(const uint8_t* win, u32 lo, uint8_t* g, u32 n) {
  const u32 lane = lane_id();
  if (n == 0) return;
  const uintptr_t ga = reinterpret_cast<uintptr_t>(g);
  const u32 head = (u32)((16 - (ga & 15)) & 15);           // bytes before the first aligned piece
  const u32 h = head < n ? head : n;
  const u32 body = (n - h) & ~15u;
  for (u32 k = lane; k < h; k += kWave) g[k] = win[lo + k];
  for (u32 k = 16 * lane; k < body; k += 16 * kWave) {
    const uint8_t* s = win + lo + h + k;
    uint4 v;
    v.x = (u32)s[0] | (u32)s[1] << 8 | (u32)s[2] << 16 | (u32)s[3] << 24;
    v.y = (u32)s[4] | (u32)s[5] << 8 | (u32)s[6] << 16 | (u32)s[7] << 24;
    v.z = (u32)s[8] | (u32)s[9] << 8 | (u32)s[10] << 16 | (u32)s[11] << 24;
    v.w = (u32)s[12] | (u32)s[13] << 8 | (u32)s[14] << 16 | (u32)s[15] << 24;
    *reinterpret_cast<uint4*>(g + h + k) = v;
  }
  for (u32 k = h + body + lane; k < n; k += kWave) g[k] = win[lo + k];
}

// Stages global bytes [s, s + n) into win[0 .. n) (byte-exact).
__device__ __forceinline__ void stage_bytes(const uint8_t* src, u64 s, u32 n, uint8_t* win) {
  const u32 lane = lane_id();
  for (u32 k = lane; k < n; k += kWave) win[k] = src[s + k];
}

// Decompresses the snappy stream in[0 .. n) into out[0 .. want). Wave-uniform control flow.
__device__ __forceinline__ bool snappy_decode(const uint8_t* in, u32 n, u32 ip, uint8_t* out,
                                              u32 want) {
  const u32 lane = lane_id();
  u32 d = 0;
  while (ip < n) {
    const u32 w0 = lds_u32(in, ip), w1 = lds_u32(in, ip + 4);
    const u32 tag = w0 & 0xFF;
    ip += 1;
    u32 len, off;
    const u32 kind = tag & 3;
    if (kind == 0) {                                          // literal
      len = (tag >> 2) + 1;
      if ((tag >> 2) >= 60) {
        const u32 nb = (tag >> 2) - 59;
        const u64 v = ((u64)w1 << 24 | (w0 >> 8)) & ((1ull << (8 * nb)) - 1);
        if (ip + nb > n || v + 1 > 0xFFFFFFFFull) return false;
        ip += nb;
        len = (u32)v + 1;
      }
      if ((u64)ip + len > n || (u64)d + len > want) return false;
      for (u32 k = lane; k < len; k += kWave) out[d + k] = in[ip + k];
      ip += len;
      d += len;
      continue;
    }
    if (kind == 1) {                                          // copy, 1-byte offset
      if (ip + 1 > n) return false;
      len = 4 + ((tag >> 2) & 7);
      off = ((tag >> 5) << 8) | ((w0 >> 8) & 0xFF);
      ip += 1;
    } else if (kind == 2) {                                   // copy, 2-byte offset
      if (ip + 2 > n) return false;
      len = 1 + (tag >> 2);
      off = (w0 >> 8) & 0xFFFF;
      ip += 2;
    } else {                                                  // copy, 4-byte offset
      if (ip + 4 > n) return false;
      len = 1 + (tag >> 2);
      off = (w0 >> 8) | (w1 << 24);
      ip += 4;
    }
    if (off == 0 || off > d || (u64)d + len > want) return false;
    // the source run precedes the copy; an overlapping copy repeats with period `off`
    for (u32 k = lane; k < len; k += kWave) out[d + k] = out[d - off + (off >= len ? k : k % off)];
    d += len;
  }
  return d == want;
}

// One block. Returns false when it does not fit the windows (the caller defers it).
template <u32 kIn, u32 kOut>
__device__ __forceinline__ bool codec_block(const CodecParams& p, u32 b, uint8_t* in,
                                            uint8_t* out, bool last_resort) {
  const u32 lane = lane_id();
  const u64 s = uni64(p.ext[b]), e = uni64(p.ext[b + 1]);
  const u64 len = e - s;
  const u64 D0 = uni64(p.dst_ext[b]), D1 = uni64(p.dst_ext[b + 1]);
  uint8_t* dst = p.dst + D0;
  const u64 dn = D1 - D0;
  const u32 tag = len ? uni(p.src[e - 1]) : 0u;
  if (len == 0 || tag != 2) {                                 // copied unchanged
    const u64 n = len < dn ? len : dn;
    for (u64 k = lane; k < n; k += kWave) dst[k] = p.src[s + k];
    if (lane == 0) p.status[b] = TPZ_BLOCK_OK;
    return true;
  }
  u64 want = 0;
  const u32 h = snappy_header(p.src + s, len - 1, want);
  bool ok = h != 0 && want + 1 == dn;
  u32 st = TPZ_BLOCK_CODEC_ERROR;
  if (ok) {
    if (len - 1 + kInSlack > kIn || want + 1 > kOut) {
      if (!last_resort) return false;
      ok = false;
      st = TPZ_BLOCK_TOO_LARGE;
    }
  } else if (h != 0 && want + 1 > TPZ_MAX_BLOCK_BYTES) {
    st = TPZ_BLOCK_TOO_LARGE;                                  // the sizes kernel gave it 1 byte
  }
  if (ok) {
    stage_bytes(p.src, s, (u32)(len - 1), in);
    __builtin_amdgcn_wave_barrier();
    ok = snappy_decode(in, (u32)(len - 1), h, out, (u32)want);
    __builtin_amdgcn_wave_barrier();
  }
  if (ok) {
    if (lane == 0) out[want] = 1;                              // re-tagged Uncompress
    __builtin_amdgcn_wave_barrier();
    store_bytes(out, 0, dst, (u32)(want + 1));
    if (lane == 0) p.status[b] = TPZ_BLOCK_OK;
  } else {
    if (lane == 0) {
      if (dn) dst[dn - 1] = 0;                                 // decodes as BAD_TAG
      p.status[b] = (uint8_t)st;
    }
  }
  __builtin_amdgcn_wave_barrier();
  return true;
}

__global__ __launch_bounds__(kWave * kSmallWaves) void codec_wave_kernel(CodecParams p) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kSmallWaves * (kSmallIn + kSmallOut)];
  const u32 wid = uni(threadIdx.x >> 6);
  uint8_t* in = lds + wid * (kSmallIn + kSmallOut);
  uint8_t* out = in + kSmallIn;
  for (u32 b = blockIdx.x * kSmallWaves + wid; b < p.n_blocks; b += gridDim.x * kSmallWaves) {
    if (!codec_block<kSmallIn, kSmallOut>(p, b, in, out, false) && lane_id() == 0)
      p.defer_list[atomicAdd(p.defer_count, 1u)] = b;
  }
}

__global__ __launch_bounds__(kWave) void codec_big_kernel(CodecParams p) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kBigIn + kBigOut];
  const u32 cnt = uni(*p.defer_count);
  for (u32 it = blockIdx.x; it < cnt; it += gridDim.x)
    codec_block<kBigIn, kBigOut>(p, uni(p.defer_list[it]), lds, lds + kBigIn, true);
}

}  // namespace

void launch_codec_sizes(const CodecLaunch& a, hipStream_t stream) {
  CodecParams p{};
  p.src = a.src;
  p.ext = a.ext;
  p.src_bytes = a.src_bytes;
  p.n_blocks = a.n_blocks;
  p.size = a.size;
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
  u32 grid = (a.n_blocks + kSmallWaves - 1) / kSmallWaves;
  if (grid > a.num_cus) grid = a.num_cus;
  if (grid == 0) grid = 1;
  hipLaunchKernelGGL(codec_wave_kernel, dim3(grid), dim3(kWave * kSmallWaves), 0, stream, p);
  hipLaunchKernelGGL(codec_big_kernel, dim3(a.num_cus), dim3(kWave), 0, stream, p);
}

}  // namespace tpz
