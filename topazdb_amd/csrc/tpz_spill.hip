// tpz_spill.hip — gfx950 kernel for the blocks the LDS decode paths hand over (the spill path).
//
// The wave and big-block paths of tpz_decode.hip stage a block in LDS and write its entries into
// the block's slot, whose size follows from the block's encoded length. Two kinds of block do
// not fit that contract, and the reference decodes both:
//   * blocks whose entries overlap or repeat: BlockIterator::seek_to (src/block/iterator.rs:
//     63-83) reads entry i at offsets[i] with no ordering or disjointness check, so n entries may
//     materialise far more bytes than the block holds;
//   * blocks longer than the LDS paths take (Block::decode, src/block.rs:46-65, has no length
//     limit; a block_size > 64 KiB builder, or a hand-made block, produces them);
//   * blocks with entries out of range: Block::decode checks no entry, so the reference returns
//     Ok(Block) and panics only when an iterator reaches such an entry (iterator.rs:74-82). These
//     are decoded with a class byte per entry (TPZ_BLOCK_BAD_ENTRY, include/tpz_gpu.h): every
//     readable key and value is materialised, and a reader fails exactly where the reference
//     does.
// Those paths append such blocks to the stream's spill worklist; this kernel decodes them into
// the caller's spill arena (include/tpz_gpu.h: TPZ_BLOCK_OK_SPILLED), straight from HBM:
//   1. compress::decode tag dispatch (src/block/compress.rs:95-113) and the CRC split
//      (src/block.rs:49-52);
//   2. CRC-32 (src/checksum.rs:6-21): every thread folds a contiguous run of 16-byte pieces
//      (slice-by-16 from LDS tables), shifts its raw CRC to the payload end with x^(8d) mod P
//      (GF(2) multiplies, square-and-multiply over x^(8*2^j)), and the workgroup XORs them;
//      the init value enters as shift_P(0xFFFFFFFF);
//   3. n and the offsets (src/block.rs:54-59), every entry's bounds checks
//      (src/block/iterator.rs:74-82) and class, and the key/value totals;
//   4. the record is reserved in the arena with one 64-bit atomic add; the entry ends are
//      written by a workgroup scan and each entry's key and value bytes are copied by one wave.
// One 1024-thread workgroup per block, persistent over the worklist. Spills are rare (no block a
// block_size <= 64 KiB BlockBuilder writes spills), so this path favours generality: any
// length, any n, any overlap.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tpz_internal.h"

namespace tpz {

// Compiled as part of tpz_decode.hip (its decode_tail_kernel runs spill_phase).
namespace sp {

typedef uint32_t u32;
typedef uint64_t u64;

constexpr int kWave = 64;
constexpr int kWaves = 16;
constexpr int kThreads = kWave * kWaves;

__device__ __forceinline__ u32 lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// a * b mod P, reflected (bit 31 = x^0), as tpz_decode.hip's gf_mul.
__device__ __forceinline__ u32 gf_mul(u32 a, u32 b) {
  u32 p = 0;
#pragma unroll
  for (int i = 0; i < 32; i++) {
    p ^= (a & (0x80000000u >> i)) ? b : 0u;
    b = (b >> 1) ^ ((b & 1u) ? 0xEDB88320u : 0u);
  }
  return p;
}

struct SpillParams {
  const uint8_t* src;
  const u64* ext;
  u64 src_bytes;
  const u32* tables;     // the decode tables; ids 0..15 = T_0..T_15 (slice-by-16)
  const u32* list;       // spill worklist
  uint8_t* spill;
  u64 spill_cap;
  u64* spill_off;
  u64* spill_used;
  u32* count;
  uint8_t* status;
  u32* crc;
  // flat layout (keys non-null, tpz_decode_blocks_flat): ends, keys and values straight into the
  // caller's columns; the arena record holds only a BAD_ENTRY block's class bytes
  u32* ends;
  const u64* efirst;
  uint8_t* keys;
  uint8_t* vals;
  const u64* kfirst;
  const u64* vfirst;
  u32 xp[64];            // x^(8 * 2^j) mod P
};

// x^(8d) mod P: the operator "append d zero bytes".
__device__ __forceinline__ u32 x8n(const SpillParams& p, u64 d) {
  u32 r = 0x80000000u;
  for (int j = 0; d; j++, d >>= 1)
    if (d & 1u) r = gf_mul(p.xp[j], r);
  return r;
}

__device__ __forceinline__ u32 be16(const uint8_t* a) { return ((u32)a[0] << 8) | a[1]; }

__device__ __forceinline__ u32 tl(const u32* tab, int id, u32 byte) { return tab[id * 256 + byte]; }

__device__ __forceinline__ u32 slice16(const u32* t, u32 w0, u32 w1, u32 w2, u32 w3) {
  return tl(t, 15, w0 & 0xFF) ^ tl(t, 14, (w0 >> 8) & 0xFF) ^ tl(t, 13, (w0 >> 16) & 0xFF) ^
         tl(t, 12, w0 >> 24) ^ tl(t, 11, w1 & 0xFF) ^ tl(t, 10, (w1 >> 8) & 0xFF) ^
         tl(t, 9, (w1 >> 16) & 0xFF) ^ tl(t, 8, w1 >> 24) ^ tl(t, 7, w2 & 0xFF) ^
         tl(t, 6, (w2 >> 8) & 0xFF) ^ tl(t, 5, (w2 >> 16) & 0xFF) ^ tl(t, 4, w2 >> 24) ^
         tl(t, 3, w3 & 0xFF) ^ tl(t, 2, (w3 >> 8) & 0xFF) ^ tl(t, 1, (w3 >> 16) & 0xFF) ^
         tl(t, 0, w3 >> 24);
}

// Workgroup reductions / scan through LDS (red: kWaves words). Every thread calls them.
__device__ __forceinline__ u64 wg_sum64(u64 x, u64* red) {
  const u32 lane = lane_id(), wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  __syncthreads();
  if (lane == 0) red[wid] = x;
  __syncthreads();
  u64 t = 0;
#pragma unroll
  for (int w = 0; w < kWaves; w++) t += red[w];
  return t;
}
__device__ __forceinline__ u32 wg_xor(u32 x, u64* red) {
  const u32 lane = lane_id(), wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x ^= __shfl_xor(x, o, 64);
  __syncthreads();
  if (lane == 0) red[wid] = x;
  __syncthreads();
  u32 t = 0;
#pragma unroll
  for (int w = 0; w < kWaves; w++) t ^= (u32)red[w];
  return t;
}
// Inclusive scan of x over the workgroup; also returns the workgroup total.
__device__ __forceinline__ u32 wg_scan(u32 x, u64* red, u32& total) {
  const u32 lane = lane_id(), wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const u32 y = __shfl_up(x, o, 64);
    if (lane >= (u32)o) x += y;
  }
  __syncthreads();
  if (lane == 63) red[wid] = x;
  __syncthreads();
  u32 before = 0, t = 0;
#pragma unroll
  for (int w = 0; w < kWaves; w++) {
    const u32 v = (u32)red[w];
    before += (u32)w < wid ? v : 0u;
    t += v;
  }
  total = t;
  return x + before;
}

// Entry i's key and value (iterator.rs:74-82): offset, the readable lengths (an unreadable key
// or value counts 0 bytes) and the entry's class (tpz_entry_class): BAD_KEY where reading the
// key panics (`data[offset..]`, get_u16, `buf[..klen]`, :74-78; seek_to_key reads no more,
// :95-98), BAD_VALUE where only the value part panics (get_u16, `buf[..vlen]`, :80-82).
struct Entry {
  u64 off;
  u32 kl, vl;
  u32 cls;
};
__device__ __forceinline__ Entry parse(const uint8_t* blk, u64 db, u64 dl, u32 i) {
  Entry e;
  e.off = be16(blk + 2 + 2 * (u64)i);                                            // :74
  e.kl = e.vl = 0;
  e.cls = TPZ_ENTRY_BAD_KEY;
  if (e.off + 2 > dl) return e;                                                  // :75-77
  const u32 kl = be16(blk + db + e.off);
  if (e.off + 2 + kl > dl) return e;                                             // :78
  e.kl = kl;
  e.cls = TPZ_ENTRY_BAD_VALUE;
  if (e.off + 4 + kl > dl) return e;                                             // :80
  const u32 vl = be16(blk + db + e.off + 2 + kl);
  if (e.off + 4 + kl + vl > dl) return e;                                        // :81-82
  e.vl = vl;
  e.cls = TPZ_ENTRY_OK;
  return e;
}

// dst[0 .. n) = src[0 .. n) by one wave; four bytes in flight per lane.
__device__ __forceinline__ void wave_copy(uint8_t* dst, const uint8_t* src, u32 n) {
  u32 k = lane_id();
  for (; k + 192 < n; k += 256) {
    const uint8_t a = src[k], b = src[k + 64], c = src[k + 128], d = src[k + 192];
    dst[k] = a;
    dst[k + 64] = b;
    dst[k + 128] = c;
    dst[k + 192] = d;
  }
  for (; k < n; k += 64) dst[k] = src[k];
}

__device__ __forceinline__ void put_meta(const SpillParams& p, u32 b, u32 st, u32 n, u32 crc) {
  if (threadIdx.x == 0) {
    p.status[b] = (uint8_t)st;
    p.count[b] = n;
    p.crc[b] = crc;
  }
}

// The phase's LDS (carved from decode_tail_kernel's buffer).
struct SpillLds {
  u32 tab[16 * 256];
  u64 red[kWaves];
  u64 shared_off;
  u32 e_kst[kThreads], e_vst[kThreads];  // this round's key/value stream starts
  u32 ticket;
};

// One spill-list entry (list position it) by the whole workgroup.
__device__ __forceinline__ void spill_block(const SpillParams& p, SpillLds& L, u32 it) {
  u32* tab = L.tab;
  u64* red = L.red;
  u32* e_kst = L.e_kst;
  u32* e_vst = L.e_vst;
  const u32 tid = threadIdx.x, wid = tid >> 6;
  const u32 b = p.list[it];
  const u64 s = p.ext[b], e = p.ext[b + 1], len = e - s;
  const uint8_t* blk = p.src + s;
  // compress::decode tag dispatch (compress.rs:95-113), the CRC split (block.rs:49-51)
  const u32 tag = len ? blk[len - 1] : 0u;
  if (len == 0 || tag == 0 || tag > 3 || tag != 1 || len - 1 < 4) {
    put_meta(p, b, len == 0 ? TPZ_BLOCK_EMPTY
                   : (tag == 0 || tag > 3) ? TPZ_BLOCK_BAD_TAG
                   : tag != 1 ? TPZ_BLOCK_UNSUPPORTED_CODEC : TPZ_BLOCK_MALFORMED, 0, 0);
    return;
  }
  const u64 P = len - 5;
  const u32 stored = (u32)blk[P] << 24 | (u32)blk[P + 1] << 16 | (u32)blk[P + 2] << 8 | blk[P + 3];

  // ---- CRC-32 of the payload [s, s + P) (checksum.rs:6-21)
  const u64 A0 = s & ~15ull, Aend = s + P;
  const u64 npc = (Aend - A0 + 15) >> 4;             // 16-byte pieces from A0
  const u64 pp = (npc + kThreads - 1) / kThreads;
  const u64 k0 = (u64)tid * pp, k1 = k0 + pp < npc ? k0 + pp : npc;
  // the thread's own descriptor starts at its first piece, so a block of any length is read
  // whole (a thread's run is npc / 1024 pieces: under 2 GiB for blocks under 2 TiB)
  const u64 T0 = A0 + 16 * k0;
  u64 rem = p.src_bytes > T0 ? p.src_bytes - T0 : 0;
  rem = rem < 0x7FFFFFF0ull ? rem : 0x7FFFFFF0ull;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(p.src + T0), (short)0, (int)rem, 0x00020000);
  u32 c = 0;
  for (u64 k = k0; k < k1; k++) {
    const u64 a = A0 + 16 * k;
    uint4 v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (u32)(16 * (k - k0)), 0, 0));
    if (a < s) {                                     // bytes before the payload: zero (a raw
      const u32 z = (u32)(s - a);                    // CRC ignores leading zeros)
      u32 w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int lo = 4 * q;
        const u32 m = (int)z >= lo + 4 ? 0u : ((int)z <= lo ? ~0u : (~0u << (8 * (z - lo))));
        w[q] &= m;
      }
      v = make_uint4(w[0], w[1], w[2], w[3]);
    }
    if (a + 16 <= Aend) {
      c = slice16(tab, v.x ^ c, v.y, v.z, v.w);
    } else {                                         // the payload's last piece
      const u32 w[4] = {v.x, v.y, v.z, v.w};
      for (u32 j = 0; j < (u32)(Aend - a); j++) {
        const u32 byte = (w[j >> 2] >> (8 * (j & 3))) & 0xFF;
        c = (c >> 8) ^ tab[(c ^ byte) & 0xFF];
      }
    }
  }
  u32 contrib = 0;
  if (k0 < k1) {
    const u64 end_t = A0 + 16 * k1 < Aend ? A0 + 16 * k1 : Aend;
    contrib = Aend == end_t ? c : gf_mul(x8n(p, Aend - end_t), c);
  }
  const u32 R = wg_xor(contrib, red);
  const u32 crc = ~(R ^ gf_mul(x8n(p, P), 0xFFFFFFFFu));
  if (crc != stored) {                                                         // checksum.rs:17
    put_meta(p, b, TPZ_BLOCK_CHECKSUM_MISMATCH, 0, crc);
    return;
  }
  // ---- n and the offsets (block.rs:54-59)
  if (P < 2) {
    put_meta(p, b, TPZ_BLOCK_MALFORMED, 0, crc);
    return;
  }
  const u32 n = be16(blk);
  if (P < 2 + 2 * (u64)n) {
    put_meta(p, b, TPZ_BLOCK_MALFORMED, 0, crc);
    return;
  }
  const u64 db = 2 + 2 * (u64)n, dl = P - db;
  // ---- pass 1: every entry's bounds (iterator.rs:74-82) and the key/value totals
  u64 kt = 0, vt = 0, bad = 0;
  for (u32 i = tid; i < n; i += kThreads) {
    const Entry en = parse(blk, db, dl, i);
    kt += en.kl;
    vt += en.vl;
    bad |= en.cls != TPZ_ENTRY_OK ? 1u : 0u;
  }
  const u64 K = wg_sum64(kt, red), V = wg_sum64(vt, red), B = wg_sum64(bad, red);
  // ---- the record: ends, then the stream (keys | values from value_start(K)), then for a
  // block with bad entries their classes (Ok(Block) either way: block.rs:46-65)
  // (flat: the columns hold the entries; a record only for the class bytes of a bad block)
  const bool flat = p.keys != nullptr;
  const u64 ncls = B ? (((u64)n + 127u) & ~127ull) : 0u;
  const u64 need = flat ? ncls : spill_record_bytes(n, K, V) + ncls;
  if (tid == 0) {
    u64 off = 0;
    if (need) {
      off = atomicAdd(reinterpret_cast<unsigned long long*>(p.spill_used), (unsigned long long)need);
      const bool fits = off + need <= p.spill_cap;
      p.spill_off[b] = fits ? off : need;
      off = fits ? off : ~0ull;
    }
    L.shared_off = off;
  }
  __syncthreads();
  const u64 roff = L.shared_off;
  if (roff == ~0ull) {
    put_meta(p, b, TPZ_BLOCK_SPILL_FULL, n, crc);
    return;
  }
  u32* ends = flat ? p.ends + 2 * p.efirst[b] : reinterpret_cast<u32*>(p.spill + roff);
  uint8_t* stream = p.spill + roff + spill_stream(n);
  uint8_t* classes = flat ? p.spill + roff : p.spill + roff + spill_record_bytes(n, K, V);
  uint8_t* kdst = flat ? p.keys + p.kfirst[b] : stream;
  uint8_t* vdst = flat ? p.vals + p.vfirst[b] : stream + value_start(K);
  u32 kc = 0, vc = 0;
  for (u32 r0 = 0; r0 < n; r0 += kThreads) {
    const u32 i = r0 + tid;
    const Entry en = i < n ? parse(blk, db, dl, i) : Entry{0, 0, 0, TPZ_ENTRY_OK};
    u32 ktot, vtot;
    const u32 ki = wg_scan(en.kl, red, ktot) + kc;
    const u32 vi = wg_scan(en.vl, red, vtot) + vc;
    if (i < n) {
      *reinterpret_cast<uint2*>(ends + 2 * (u64)i) = make_uint2(ki, vi);
      if (B) classes[i] = (uint8_t)en.cls;
      e_kst[tid] = ki - en.kl;
      e_vst[tid] = vi - en.vl;
    }
    __syncthreads();
    // one wave per entry: its key, then its value (src/block/iterator.rs:78-82)
    const u32 m = n - r0 < (u32)kThreads ? n - r0 : (u32)kThreads;
    for (u32 j = wid; j < m; j += kWaves) {
      const Entry ej = parse(blk, db, dl, r0 + j);
      wave_copy(kdst + e_kst[j], blk + db + ej.off + 2, ej.kl);
      wave_copy(vdst + e_vst[j], blk + db + ej.off + 4 + ej.kl, ej.vl);
    }
    kc += ktot;
    vc += vtot;
    __syncthreads();
  }
  put_meta(p, b, B ? TPZ_BLOCK_BAD_ENTRY : flat ? TPZ_BLOCK_OK : TPZ_BLOCK_OK_SPILLED, n, crc);
}

// Phase C of decode_tail_kernel (tpz_decode.hip): the cnt blocks of the spill list, one per
// workgroup, claimed from the ticket counter. Every thread of the workgroup calls it.
__device__ __forceinline__ void spill_phase(const SpillParams& p, uint8_t* lds_bytes, u32 cnt,
                                            u32* ticket) {
  SpillLds& L = *reinterpret_cast<SpillLds*>(lds_bytes);
  u32* tab = L.tab;
  u64* red = L.red;
  const u32 tid = threadIdx.x, lane = lane_id(), wid = tid >> 6;
  for (u32 i = tid; i < 16 * 256; i += kThreads) tab[i] = p.tables[i];

  for (;;) {
    __syncthreads();                                  // the previous block's LDS reads are done
    if (tid == 0) L.ticket = atomicAdd(ticket, 1u);
    __syncthreads();
    const u32 it = __builtin_amdgcn_readfirstlane(L.ticket);
    if (it >= cnt) break;
    spill_block(p, L, it);
  }
  (void)lane;
  (void)wid;
}

SpillParams spill_params(const SpillLaunch& a) {
  SpillParams p{};
  p.src = a.src;
  p.ext = a.ext;
  p.src_bytes = a.src_bytes;
  p.tables = a.crc_tables;
  p.list = a.list;
  p.spill = a.spill;
  p.spill_cap = a.spill ? a.spill_cap : 0;
  p.spill_off = a.spill_off;
  p.spill_used = a.spill_used;
  p.count = a.count;
  p.status = a.status;
  p.crc = a.crc;
  p.ends = a.ends;
  p.efirst = a.efirst;
  p.keys = a.keys;
  p.vals = a.vals;
  p.kfirst = a.kfirst;
  p.vfirst = a.vfirst;
  // x^(8 * 2^j) mod P by repeated squaring, from x^8
  u32 x = 0x80000000u >> 8;
  for (int j = 0; j < 64; j++) {
    p.xp[j] = x;
    // square: x * x mod P (host restatement of gf_mul)
    u32 a2 = x, b2 = x, r = 0;
    for (int i = 0; i < 32; i++) {
      r ^= (a2 & (0x80000000u >> i)) ? b2 : 0u;
      b2 = (b2 >> 1) ^ ((b2 & 1u) ? 0xEDB88320u : 0u);
    }
    x = r;
  }
  return p;
}

}  // namespace sp
}  // namespace tpz
