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

// ------------------------------------------------------------------ open -> flat layout, one read
// tpz_verify_files_flat_layout: FileObject::open's whole-file CRC (src/table/file_object.rs:57-78)
// of every SST file and tpz_flat_layout's per-block reservations of its data blocks from ONE read
// of the blocks (the reference's open reads every byte of the file for the CRC before any block is
// read, src/table.rs:91-112; the flat decode reads them again).
//
// The blocks are the decode's batch (every file's data region, back to back in one buffer); the
// rest of each file (meta, bloom, offsets and the CRC trailer: its "tail") lies in a second batch.
// Raw CRCs R0 (init 0, no xorout) are linear: R0(A || B) = Z_|B|(R0(A)) ^ R0(B). File f is
// data_f || tail_f and its CRC region all but the last 4 bytes, so
//   R0(region) = Z_{|tail| - 4}(D) ^ R0(tail[..-4]),  D = XOR over its blocks b of Z_{dend - e_b}(R0(b))
// (dend = the end of the file's data region).
// open_blocks_kernel (one wave per block at a time, persistent): the block is staged in the wave's
// LDS window (as flat_sizes_kernel), parsed for its reservation, and folded: lane l takes the
// 80-byte run that ends 80 l bytes before the block's end rounded up to 16 (bytes outside the block
// read as zero: leading zeros leave R0 unchanged, the k trailing ones give Z_k(R0(b))), slice-by-16
// in LDS, shifted by 80 l with a per-lane GF(2) multiply, XORed over the wave. Long blocks fold
// 5120-byte rounds straight from HBM. open_finish_kernel (one workgroup per file) shifts every
// block's value to the end of the file's data region (a thread per block: a GF(2) multiply by
// x^(8 n) from byte-indexed power tables, no dependent chain of shift operators), XORs them, folds
// the rest of the file, applies the init term and compares with the trailer. (A first version
// shifted each block in the blocks kernel with the shift-by-16*2^j operators: ~22 dependent
// global lookups per block, 2.32 ms for the 4k shard.)
constexpr int kOpWaves = 8;
constexpr int kOpThreads = kOpWaves * 64;
constexpr int kOpGuard = 96;                      // zeroed: a lane run may start up to 80 B before 0
constexpr int kOpSlot = kOpGuard + kFlWin;
constexpr int kOpTabBytes = 16 * 1024;       // slice-by-16 (conflict-light replicated layouts:
constexpr int kOpWgsPerCu = 3;                // slower)
constexpr int kOpLds = kOpTabBytes + kOpWaves * kOpSlot;

// A wave-uniform 64-bit value loaded by a vector load, made visibly uniform (readfirstlane):
// buffer descriptors built from it stay in SGPRs (otherwise the compiler wraps every buffer load
// in a waterfall loop over the lanes' descriptors).
// (readfirstlane returns int: each half goes through a u32, or the low half would be
// sign-extended into the high one for offsets of 2 GiB and more)
__device__ __forceinline__ u64 op_uni64(u64 x) {
  const u32 lo = __builtin_amdgcn_readfirstlane((u32)x), hi = __builtin_amdgcn_readfirstlane((u32)(x >> 32));
  return ((u64)hi << 32) | lo;
}

struct OpenParams {
  const uint8_t* src;
  const u64* bext;        // the blocks: block b = src[bext[b] .. bext[b + 1])
  u64 src_bytes;
  u32 nb;
  const u32* fblock;      // file f's blocks: fblock[f] .. fblock[f + 1] - 1 (nf + 1 entries)
  u32 nf;
  const uint8_t* tsrc;    // the tails: tail f = tsrc[text[f] .. text[f + 1])
  const u64* text;
  u64* first;             // 3 x (nb + 1): reservations (scanned afterwards)
  u32* cb;                // nb: Z_{k_b}(R0(block b)) (open_blocks_kernel)
  const u32* tacc;        // nf: R0 of each tail's main part (crc_window_kernel, trailer 4)
  const u32* dtab;        // the decode tables (ids 0..15 slice-by-16, kCrcInvTable)
  const u32* rtab;        // the range tables (shift-by-16*2^j operators)
  u32* crc;               // nf
  uint8_t* status;        // nf
  u32 lane_shift[64];     // x^(8 * 80 l) mod P
  u32 round_shift;        // x^(8 * 5120) mod P
};

__device__ __forceinline__ u32 op_xor3(u32 a, u32 b, u32 c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
// R0 of one 16-byte chunk (w0..w3 little-endian) after the register value folded into w0.
__device__ __forceinline__ u32 op_slice16(const u32* t, u32 w0, u32 w1, u32 w2, u32 w3) {
  u32 c = op_xor3(t[15 * 256 + (w0 & 0xFF)], t[14 * 256 + ((w0 >> 8) & 0xFF)], t[13 * 256 + ((w0 >> 16) & 0xFF)]);
  c = op_xor3(c, t[12 * 256 + (w0 >> 24)], t[11 * 256 + (w1 & 0xFF)]);
  c = op_xor3(c, t[10 * 256 + ((w1 >> 8) & 0xFF)], t[9 * 256 + ((w1 >> 16) & 0xFF)]);
  c = op_xor3(c, t[8 * 256 + (w1 >> 24)], t[7 * 256 + (w2 & 0xFF)]);
  c = op_xor3(c, t[6 * 256 + ((w2 >> 8) & 0xFF)], t[5 * 256 + ((w2 >> 16) & 0xFF)]);
  c = op_xor3(c, t[4 * 256 + (w2 >> 24)], t[3 * 256 + (w3 & 0xFF)]);
  c = op_xor3(c, t[2 * 256 + ((w3 >> 8) & 0xFF)], t[1 * 256 + ((w3 >> 16) & 0xFF)]);
  return c ^ t[w3 >> 24];
}
// a * b mod P, reflected (bit 31 = x^0), per lane.
__device__ __forceinline__ u32 op_gfmul(u32 a, u32 b) {
  u32 p = 0;
#pragma unroll
  for (int i = 0; i < 32; i++) {
    p ^= b & (u32)((int)(a << i) >> 31);
    b = (b >> 1) ^ (0xEDB88320u & (u32)(-(int)(b & 1u)));
  }
  return p;
}
__device__ __forceinline__ u32 op_wave_xor(u32 x) {
  for (u32 o = 1; o < 64; o <<= 1) x ^= __shfl_xor(x, o, 64);
  return x;
}
// Z_n(a) from the range tables: the n mod 16 bytes with the slice tables, then the shift-by-16*2^j
// operators for the bits of n / 16.
__device__ __forceinline__ u32 op_zshift(const u32* g, u32 a, u64 n) {
  const u32 k = (u32)(n & 15);
  if (k) {
    u32 r = k >= 4 ? 0u : (a >> (8 * k));
    for (u32 i = 0; i < 4 && i < k; i++) r ^= g[(k - 1 - i) * 256 + ((a >> (8 * i)) & 0xFF)];
    a = r;
  }
  u64 m = n >> 4;
  for (int j = 0; m; j++, m >>= 1)
    if (m & 1) {
      const u32* t = g + (16 + 4 * j) * 256;
      a = op_xor3(t[a & 0xFF], t[256 + ((a >> 8) & 0xFF)], t[512 + ((a >> 16) & 0xFF)]) ^ t[768 + (a >> 24)];
    }
  return a;
}
// The inverse of Z_k for k < 16: un-feed k zero bytes (the decode tables' T_0 and inverse table).
__device__ __forceinline__ u32 op_unshift(const u32* d, u32 r, u32 k) {
  for (u32 i = 0; i < k; i++) {
    const u32 b = d[kCrcInvTable * 256 + (r >> 24)];
    r = ((r ^ d[b]) << 8) | b;
  }
  return r;
}
// 16 bytes of the message at absolute offset x (16-aligned) with the bytes outside [lo, hi) zeroed;
// no byte outside [lo, hi) is read (a chunk that [lo, hi) cuts is read byte by byte).
__device__ __forceinline__ uint4 op_chunk(const uint8_t* src, int64_t x, u64 lo, u64 hi) {
  if (x + 16 <= (int64_t)lo || x >= (int64_t)hi) return make_uint4(0, 0, 0, 0);
  if (x >= (int64_t)lo && x + 16 <= (int64_t)hi) return *reinterpret_cast<const uint4*>(src + x);
  u32 w[4] = {0, 0, 0, 0};
  for (int i = 0; i < 16; i++) {
    const int64_t a = x + i;
    if (a >= (int64_t)lo && a < (int64_t)hi) w[i >> 2] |= (u32)src[a] << (8 * (i & 3));
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

__global__ __launch_bounds__(kOpThreads) void open_blocks_kernel(OpenParams p) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kOpLds];
  u32* tab = reinterpret_cast<u32*>(lds);
  for (int i = threadIdx.x; i < 16 * 256 / 4; i += kOpThreads)
    reinterpret_cast<uint4*>(tab)[i] = reinterpret_cast<const uint4*>(p.dtab)[i];
  auto fold = [&](u32 c, const uint4& w) { return op_slice16(tab, w.x ^ c, w.y, w.z, w.w); };
  const u32 lane = lane_id(), wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* slot = lds + kOpTabBytes + wid * kOpSlot;
  uint8_t* win = slot + kOpGuard;
  if (lane < kOpGuard / 16) reinterpret_cast<uint4*>(slot)[lane] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  const u32 kl = p.lane_shift[lane];
  const u64 st = (u64)p.nb + 1;
  const u64 V = (u64)gridDim.x * kOpWaves;
  // blocks v, v + V, ...: the waves of the grid on adjacent blocks at a time
  // the next block's pieces are loaded while the current one is parsed and folded (staged
  // blocks: lengths up to kFlMaxLen whose last piece lies inside src_bytes)
  auto staged = [&](u64 s, u64 e) { return e > s && e - s <= kFlMaxLen && ((e + 15) & ~15ull) <= p.src_bytes; };
  uint4 v[kFlRounds];
  auto issue = [&](u64 s, u64 e) {
    const __amdgpu_buffer_rsrc_t rs = src_rsrc(p.src, (e + 15) & ~15ull, s & ~15ull);
#pragma unroll
    for (int r = 0; r < kFlRounds; r++)
      v[r] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (u32)(r * 1024 + lane * 16), 0, 0));
  };
  u64 b = (u64)blockIdx.x * kOpWaves + wid;
  u64 s = 0, e = 0;
  if (b < p.nb) {
    s = op_uni64(p.bext[b]);
    e = op_uni64(p.bext[b + 1]);
    if (staged(s, e)) issue(s, e);
  }
  for (; b < p.nb; b += V) {
    const bool stg = staged(s, e);
    if (stg) {
#pragma unroll
      for (int r = 0; r < kFlRounds; r++)
        if (r * 1024 + lane * 16 < (u32)kFlWin) *reinterpret_cast<uint4*>(win + r * 1024 + lane * 16) = v[r];
    }
    // the next block: its extents, then its pieces
    const u64 bn = b + V;
    u64 sn = 0, en = 0;
    if (bn < p.nb) {
      sn = op_uni64(p.bext[bn]);
      en = op_uni64(p.bext[bn + 1]);
      if (staged(sn, en)) issue(sn, en);
    }
    Sizes z{0, 0, 0};
    u32 X = 0, k = 0;
    (void)k;
    if (e > s) {
      const u64 len = e - s;
      const u64 e16 = (e + 15) & ~15ull;
      // (a buffer load of a 16-byte piece that the descriptor cuts returns zeros: a block whose
      // last piece runs past src_bytes is read from HBM piece by piece, as the long ones are)
      if (stg) {
        __builtin_amdgcn_wave_barrier();
        const u32 a0 = (u32)(s & 15u), E = a0 + (u32)len, E16 = (E + 15) & ~15u;
        k = E16 - E;
        if (lane < a0) win[lane] = 0;        // the previous block's tail
        if (lane < k) win[E + lane] = 0;     // the next block's head
        __builtin_amdgcn_wave_barrier();
        z = block_sizes(win + a0, len);
        const int r0 = (int)E16 - 80 * (int)(lane + 1);
        u32 c = 0;
        if (r0 + 80 > 0) {
#pragma unroll
          for (int t = 0; t < 5; t++) {
            const uint4 w = *reinterpret_cast<const uint4*>(win + r0 + 16 * t);
            c = fold(c, w);
          }
        }
        X = op_wave_xor(op_gfmul(kl, c));
      } else {
        z = block_sizes(p.src + s, len);   // long blocks: parsed and folded from HBM
        k = (u32)(e16 - e);
        const u64 rounds = (e16 - (s & ~15ull) + 5119) / 5120;
        u32 A = 0;
        for (u64 r = rounds; r-- > 0;) {
          const int64_t r0 = (int64_t)e16 - 5120 * (int64_t)r - 80 * (int64_t)(lane + 1);
          u32 c = 0;
#pragma unroll
          for (int t = 0; t < 5; t++) {
            const uint4 w = op_chunk(p.src, r0 + 16 * t, s, e);
            c = fold(c, w);
          }
          A = op_gfmul(p.round_shift, A) ^ c;   // Horner by one 5120-byte round
        }
        X = op_wave_xor(op_gfmul(kl, A));
      }
    }
    // X = Z_k(R0(block)), k = the block's end to the next 16-byte boundary (recomputed from the
    // extent by open_finish_kernel, which shifts X to the end of the file's data region)
    if (lane == 0) {
      p.cb[b] = X;
      p.first[b] = z.n;
      p.first[st + b] = z.k;
      p.first[2 * st + b] = z.v;
    }
    __builtin_amdgcn_wave_barrier();   // (the window is restaged next)
    s = sn;
    e = en;
  }
}

// One workgroup per file: the XOR of its blocks' values, its tail's R0 (crc_window_kernel's main
// part, then the last < 16 bytes), the init term, the trailer compare (crc_finish_kernel's
// outcome; a file shorter than 4 bytes is MALFORMED, file_object.rs:69). (A first version folded
// the tails here, one workgroup per 1 MiB tail: 0.29 ms of the open for the 4k shard.)
constexpr int kFinThreads = 1024;
__global__ __launch_bounds__(kFinThreads) void open_finish_kernel(OpenParams p) {
  __shared__ u32 red[kFinThreads / 64];
  const u32 f = blockIdx.x, t = threadIdx.x;
  const u32 b0 = p.fblock[f], b1 = p.fblock[f + 1];
  const u64 dlo = p.nb ? p.bext[b0] : 0, dend = p.nb ? p.bext[b1] : 0;
  const u64 tlo = p.text[f], thi = p.text[f + 1];
  if (thi < tlo + 4) {       // (shorter than the trailer; with blocks: outside the contract)
    if (t == 0) {
      p.crc[f] = 0;
      p.status[f] = TPZ_BLOCK_MALFORMED;
    }
    return;
  }
  const u64 e = thi - 4;     // the tail's CRC bytes [tlo, e)
  // D = XOR over the file's blocks of Z_{dend - e_b}(R0(b)), one block per thread at a time:
  // X_b = Z_{k_b}(R0(b)) times x^(8 n) mod P, n = dend - e_b - k_b, the factor from the four
  // power tables (bytes of n); a block that ends less than k_b bytes before dend (the last one)
  // is un-shifted instead
  const u32* pw = p.rtab + kPowTable * 256;
  u32 D = 0;
  for (u32 b = b0 + t; b < b1; b += kFinThreads) {
    const u64 eb = p.bext[b + 1], d = dend - eb;
    const u32 kb = (u32)(((eb + 15) & ~15ull) - eb);
    const u32 X = p.cb[b];
    u32 C;
    if (d < kb) {
      C = op_unshift(p.dtab, X, kb - (u32)d);
    } else if ((d - kb) >> 32) {
      C = op_zshift(p.rtab, X, d - kb);        // (data regions of 4 GiB or more)
    } else {
      const u32 n = (u32)(d - kb);
      C = X;
#pragma unroll
      for (int i = 0; i < 4; i++)
        if ((n >> (8 * i)) & 0xFF) C = op_gfmul(pw[i * 256 + ((n >> (8 * i)) & 0xFF)], C);
    }
    D ^= C;
  }
  D = op_wave_xor(D);
  if ((t & 63) == 0) red[t >> 6] = D;
  __syncthreads();
  if (t == 0) {
    D = 0;
    for (int i = 0; i < kFinThreads / 64; i++) D ^= red[i];
    // the tail's CRC bytes [tlo, e): crc_window_kernel's R0 of the main part [tlo, A),
    // A = max(tlo, e & ~15), then the (< 16) bytes [A, e) one at a time (crc_finish_kernel)
    const u64 A = (e & ~15ull) > tlo ? (e & ~15ull) : tlo;
    u32 T = p.tacc[f];
    for (u64 x = A; x < e; x++) T = (T >> 8) ^ p.dtab[(T ^ p.tsrc[x]) & 0xFF];
    const u64 len = (dend - dlo) + (e - tlo);
    const u32 R = op_zshift(p.rtab, D, e - tlo) ^ T ^ op_zshift(p.rtab, 0xFFFFFFFFu, len);
    const u32 crc = ~R;
    p.crc[f] = crc;
    const uint8_t* tr = p.tsrc + e;     // the trailer: big-endian u32 (file_object.rs:69)
    const u32 stored = ((u32)tr[0] << 24) | ((u32)tr[1] << 16) | ((u32)tr[2] << 8) | tr[3];
    p.status[f] = crc == stored ? TPZ_BLOCK_OK : TPZ_BLOCK_CHECKSUM_MISMATCH;   // checksum.rs:17
  }
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

static u32 op_pow_shift(u64 nbytes) {   // x^(8 n) mod P, reflected (x^0 = 0x80000000)
  u32 x = 0x80000000u;
  for (u64 i = 0; i < 8 * nbytes; i++) x = (x >> 1) ^ ((x & 1u) ? 0xEDB88320u : 0u);
  return x;
}

void launch_open_flat(const OpenLaunch& a, hipStream_t stream) {
  OpenParams p;
  p.src = a.src;
  p.bext = a.bext;
  p.src_bytes = a.src_bytes;
  p.nb = a.n_blocks;
  p.fblock = a.fblock;
  p.nf = a.n_files;
  p.tsrc = a.tsrc;
  p.text = a.text;
  p.first = a.first;
  p.cb = a.cb;
  p.dtab = a.dtab;
  p.rtab = a.rtab;
  p.crc = a.crc;
  p.status = a.status;
  p.tacc = a.tacc;
  static const struct Shifts {
    u32 lane[64], round;
    Shifts() {
      for (int l = 0; l < 64; l++) lane[l] = op_pow_shift(80ull * l);
      round = op_pow_shift(5120);
    }
  } sh;
  for (int l = 0; l < 64; l++) p.lane_shift[l] = sh.lane[l];
  p.round_shift = sh.round;
  if (a.n_blocks) {
    u64 wgs = ((u64)a.n_blocks + kOpWaves - 1) / kOpWaves;
    const u64 cap = (u64)kOpWgsPerCu * a.num_cus;   // 8-wave workgroups per CU the LDS holds
    if (wgs > cap) wgs = cap;
    hipLaunchKernelGGL(open_blocks_kernel, dim3((u32)wgs), dim3(kOpThreads), 0, stream, p);
    const u32 np = (a.n_blocks + kScWg - 1) / kScWg;
    hipLaunchKernelGGL(flat_scan_parts, dim3(np, 3), dim3(256), 0, stream, a.first, a.n_blocks, a.part, np);
    hipLaunchKernelGGL(flat_scan_totals, dim3(3), dim3(1024), 0, stream, a.part, np);
    hipLaunchKernelGGL(flat_scan_write, dim3(np, 3), dim3(256), 0, stream, a.first, a.n_blocks, a.part, np);
  } else {
    (void)hipMemsetAsync(a.first, 0, 3 * 8, stream);
  }
  if (a.n_files) {
    // the tails' main parts by the whole-file CRC kernel (trailer 4: [tlo, thi - 4))
    CrcLaunch c{};
    c.src = a.tsrc;
    c.ext = a.text;
    c.src_bytes = a.tail_bytes;
    c.n_ranges = a.n_files;
    c.trailer = 4;
    c.tables = a.rtab;
    c.rep = a.rep;
    c.acc = a.tacc;
    c.num_cus = a.num_cus;
    c.acc_only = true;
    launch_crc_ranges(c, stream);
    hipLaunchKernelGGL(open_finish_kernel, dim3(a.n_files), dim3(kFinThreads), 0, stream, p);
  }
}

}  // namespace tpz
