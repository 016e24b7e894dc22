// tpz_seek.hip — gfx950 kernels for the batched point-get side of an SSTable (SURVEY.md §8f
// row 4), over a table whose blocks tpz_decode_blocks has decoded into the slotted columns.
//
//   seek_kernel   SsTableIterator::seek_to_key (src/table/iterator.rs:44-72, 74-79): for every
//                 query key, find_block_idx (src/table.rs:178-182: partition_point(first_key <=
//                 key) - 1, saturating), BlockIterator::seek_to_key in that block
//                 (src/block/iterator.rs:91-109: binary search, an equal key returns at once, else
//                 the lower bound), and, when the block iterator is invalid and a next block
//                 exists, seek_to_first of the next block.
//   bloom_kernel  SsTable::may_contain (src/table.rs:114-119) = Bloom::may_contain
//                 (src/bloom.rs:72-84) of xxh3_64(key) (xxhash-rust 0.8.5).
//
// One thread per query: both are a few binary-search steps of dependent global loads (keys of a
// few tens of bytes), latency-bound, so the launch simply puts many queries in flight. A query
// whose block did not decode gets that block's status (the reference's read_block_cached Err, or
// its panic for MALFORMED); OK_SPILLED and BAD_ENTRY blocks are read from their spill records and
// report OK, unless the seek reads an entry of a BAD_ENTRY block the reference panics on (the
// key of a BAD_KEY entry in the bisection, or any bad entry it lands on): MALFORMED.

#if defined(TPZ_BLOOM_ABL_BLOOMBYTES)   // diagnostic: the byte-load xxh3 reads
#define TPZ_XXH3_BYTEREADS
#endif
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdlib>

#include "tpz_internal.h"
#include "tpz_xxh3.h"

namespace tpz {

namespace {

typedef uint32_t u32;
typedef uint64_t u64;

// memcmp then length, as Rust's Ord for [u8]
__device__ __forceinline__ int key_cmp(const uint8_t* a, u64 al, const uint8_t* b, u64 bl) {
  const u64 n = al < bl ? al : bl;
  for (u64 i = 0; i < n; i++) {
    const u32 x = a[i], y = b[i];
    if (x != y) return x < y ? -1 : 1;
  }
  return al < bl ? -1 : (al > bl ? 1 : 0);
}

struct SeekParams {
  const uint8_t* fk;        // block first keys, packed
  const u64* fk_pos;        // n_blocks + 1
  u32 n_blocks;
  const u64* ext;           // the data region's block extents (slot bases)
  const uint8_t* data;      // decoded columns
  const u32* ends;
  const u32* count;
  const uint8_t* bstatus;
  const uint8_t* spill;     // spill arena + record offsets (OK_SPILLED blocks)
  const u64* spill_off;
  const uint8_t* q;         // query keys, packed
  const u64* q_pos;         // n_q + 1
  u32 n_q;
  u32* out_block;
  u32* out_entry;
  uint8_t* out_status;
  uint8_t* out_valid;
  const u64* efirst;        // exact ends layout, or null: slotted
};

// A decoded block's ends and stream: its slot, or its spill record (include/tpz_gpu.h); the
// entry classes of a BAD_ENTRY block (null otherwise: every entry reads whole).
struct BlockView {
  const u32* ends;
  const uint8_t* stream;
  const uint8_t* cls;
  // seek_to(j) / the bisection's key read panic on entry j (iterator.rs:74-82, :95-98)
  __device__ __forceinline__ bool seek_panics(u32 j) const { return cls && cls[j] != TPZ_ENTRY_OK; }
  __device__ __forceinline__ bool key_panics(u32 j) const { return cls && cls[j] == TPZ_ENTRY_BAD_KEY; }
};
__device__ __forceinline__ BlockView block_view(const SeekParams& p, u32 b, u32 st) {
  if (block_in_spill(st)) {
    const u32 n = p.count[b];
    const uint8_t* r = p.spill + p.spill_off[b];
    const u32* e = reinterpret_cast<const u32*>(r);
    const uint8_t* cls = (st == TPZ_BLOCK_BAD_ENTRY && n)
                             ? r + spill_classes(n, e[2 * (n - 1)], e[2 * (n - 1) + 1]) : nullptr;
    return BlockView{e, r + spill_stream(n), cls};
  }
  const u64 e0 = p.ext[b];
  return BlockView{p.ends + 2 * ends_base(p.efirst, e0, b), p.data + slot_base(e0, b), nullptr};
}
// Entry j's key: its bytes and length.
__device__ __forceinline__ const uint8_t* entry_key(const BlockView& v, u32 j, u64& len) {
  const u32 lo = j ? v.ends[2 * (j - 1)] : 0u, hi = v.ends[2 * j];
  len = hi - lo;
  return v.stream + lo;
}
__device__ __forceinline__ bool decoded(u32 st) { return block_decoded(st); }

__global__ __launch_bounds__(256) void seek_kernel(SeekParams p) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n_q) return;
  const uint8_t* qk = p.q + p.q_pos[i];
  const u64 ql = p.q_pos[i + 1] - p.q_pos[i];
  if (p.n_blocks == 0) {                      // block_metas[0]: the reference panics
    p.out_block[i] = 0;
    p.out_entry[i] = 0;
    p.out_status[i] = TPZ_BLOCK_MALFORMED;
    p.out_valid[i] = 0;
    return;
  }
  // find_block_idx: partition_point(first_key <= key) (the lower-bound bisection), minus one
  u32 lo = 0, hi = p.n_blocks;
  while (lo < hi) {
    const u32 mid = lo + (hi - lo) / 2;
    const u64 a = p.fk_pos[mid];
    if (key_cmp(p.fk + a, p.fk_pos[mid + 1] - a, qk, ql) <= 0) lo = mid + 1; else hi = mid;
  }
  u32 b = lo ? lo - 1 : 0;
  u32 st = p.bstatus[b], pos = 0;
  bool valid = false, panic = false;
  if (decoded(st)) {
    // BlockIterator::seek_to_key
    const BlockView v = block_view(p, b, st);
    const u32 n = p.count[b];
    u32 l = 0, r = n;
    pos = n;
    bool found = false;
    while (l < r) {
      const u32 mid = (r - l) / 2 + l;
      if (v.key_panics(mid)) { pos = mid; panic = true; break; }   // iterator.rs:95-98
      u64 kl;
      const uint8_t* k = entry_key(v, mid, kl);
      const int c = key_cmp(k, kl, qk, ql);
      if (c > 0) r = mid;
      else if (c < 0) l = mid + 1;
      else { pos = mid; found = true; break; }
    }
    if (!found && !panic) pos = l;
    if (!panic && pos < n && v.seek_panics(pos)) panic = true;      // seek_to, :74-82
    u64 kl = 0;
    if (pos < n) entry_key(v, pos, kl);
    valid = !panic && pos < n && kl > 0;      // is_valid: the current key is non-empty
    if (!panic && !valid && b + 1 < p.n_blocks) {   // the next block, from its first entry
      b++;
      st = p.bstatus[b];
      pos = 0;
      valid = false;
      if (decoded(st) && p.count[b] > 0) {
        const BlockView w = block_view(p, b, st);
        panic = w.seek_panics(0);
        entry_key(w, 0, kl);
        valid = !panic && kl > 0;
      }
    }
  }
  p.out_block[i] = b;
  p.out_entry[i] = pos;
  p.out_status[i] = panic ? (uint8_t)TPZ_BLOCK_MALFORMED
                          : decoded(st) ? (uint8_t)TPZ_BLOCK_OK : (uint8_t)st;
  p.out_valid[i] = decoded(st) && valid;
}

struct BloomParams {
  const uint8_t* filter;    // Bloom::encode: the bit array, then k in the last byte
  u64 filter_len;
  const uint8_t* q;
  const u64* q_pos;
  u32 n_q;
  uint8_t* out;
};

__global__ __launch_bounds__(256) void bloom_kernel(BloomParams p) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n_q) return;
  const u64 a = p.q_pos[i];
  u64 h = xxh3::hash64(p.q + a, p.q_pos[i + 1] - a);
  if (p.filter_len == 0) {                    // filter.last().unwrap() panics
    p.out[i] = 2;
    return;
  }
  const u64 delta = (h >> 34) | (h << 30);
  const u32 k = p.filter[p.filter_len - 1];
  const u64 limit = (p.filter_len - 1) * 8;
  if (limit == 0) {                           // no bit array: `% 0` panics unless k == 0
    p.out[i] = k ? 2 : 1;
    return;
  }
  uint8_t hit = 1;
  for (u32 j = 0; j < k; j++) {
    const u64 bit = h % limit;
    if (!(p.filter[bit >> 3] & (1u << (bit & 7)))) {
      hit = 0;
      break;
    }
    h += delta;
  }
  p.out[i] = hit;
}

// Bloom::from_keys (src/bloom.rs:48-70) for keys on the device: one thread per key sets its k
// probe bits (h + j * rotr(h, 34) mod limit) with 32-bit atomic ORs into the zeroed bit array
// (the geometry, limit and k, comes from the host: tpz_bloom_geometry).
__global__ __launch_bounds__(256) void bloom_build_kernel(BloomBuildLaunch a) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n_keys) return;
  const u64 s = a.key_pos[i];
  u64 h = xxh3::hash64(a.keys + s, a.key_pos[i + 1] - s);
  const u64 delta = (h >> 34) | (h << 30);                  // Bloom::delta
  u32* words = reinterpret_cast<u32*>(a.filter);
  for (u32 j = 0; j < a.k; j++) {
    const u64 bit = h % a.limit;
#if defined(TPZ_BLOOM_ABL_BLOOMWG)      // diagnostic: workgroup-scope atomics (wrong across WGs)
    __hip_atomic_fetch_or(&words[bit >> 5], 1u << (bit & 31), __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_WORKGROUP);
#elif defined(TPZ_BLOOM_ABL_BLOOMSTORE) // diagnostic: plain stores (wrong filter)
    words[bit >> 5] = 1u << (bit & 31);
#else
    atomicOr(&words[bit >> 5], 1u << (bit & 31));           // bit_set: byte bit/8, bit bit%8
#endif
    h += delta;
  }
}

// The partitioned build (filters of <= kBloomMaxSlices slices of 2^19 bits, 64 MiB): the probes are
// bucketed by slice (count, scan, scatter: LDS histograms and LDS rank counters, no global
// atomics), then a workgroup per slice ORs its bucket into a 64 KiB LDS slice and writes it out
// with plain stores. The atomic kernel above spends ~4 ms on 107 M device-scope atomics for
// 35.6 M keys; this moves ~2.6 GB instead.
constexpr uint32_t kBloomSliceLog = 19, kBloomSliceBits = 1u << kBloomSliceLog;   // 64 KiB
constexpr uint32_t kBloomMaxSlices = 1024;          // scatter LDS: 2 S words + 48 KiB <= 64 KiB

constexpr uint32_t kBloomWgProbes = 12288;         // a workgroup's probes staged in LDS (48 KiB)

// keys per workgroup: as many as keep its probes within kBloomWgProbes
__host__ __device__ inline uint32_t bloom_part_per_wg(uint32_t k) { return kBloomWgProbes / k; }
__host__ __device__ inline uint32_t bloom_part_wgs(uint32_t n, uint32_t k) {
  const uint32_t per = bloom_part_per_wg(k);
  const uint32_t w = (n + per - 1) / per;
  return w < 1 ? 1 : w;
}

struct BloomPart {
  const uint8_t* keys;
  const uint64_t* key_pos;
  uint32_t n_keys, k;
  uint64_t limit;
  uint32_t S, nwg, per_wg;
  uint32_t* hist;     // S x nwg, slice-major: the workgroups' probe counts
  uint32_t* off;      // S x nwg: their exclusive prefix within the slice
  uint32_t* tot;
  uint32_t* base;
  uint32_t* pos;
  uint32_t* words;
  uint64_t filter_words;
  uint32_t* stage;    // gather path: nwg x kBloomWgProbes, each workgroup's probes grouped by slice
};

__device__ __forceinline__ void bloom_count_pass(const BloomPart& p, uint32_t* cnt) {
  const uint64_t i0 = (uint64_t)blockIdx.x * p.per_wg;
  const uint64_t i1 = min((uint64_t)p.n_keys, i0 + p.per_wg);
  for (uint64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const uint64_t s = p.key_pos[i];
    uint64_t h = xxh3::hash64(p.keys + s, p.key_pos[i + 1] - s);
    const uint64_t delta = (h >> 34) | (h << 30);   // Bloom::delta
    for (uint32_t j = 0; j < p.k; j++) {
      atomicAdd(&cnt[(uint32_t)((h % p.limit) >> kBloomSliceLog)], 1u);   // LDS
      h += delta;
    }
  }
}

__global__ __launch_bounds__(256) void bloom_count_kernel(BloomPart p) {
  extern __shared__ uint32_t cnt[];
  for (uint32_t s = threadIdx.x; s < p.S; s += blockDim.x) cnt[s] = 0;
  __syncthreads();
  bloom_count_pass(p, cnt);
  __syncthreads();
  for (uint32_t s = threadIdx.x; s < p.S; s += blockDim.x) p.hist[(uint64_t)s * p.nwg + blockIdx.x] = cnt[s];
}

// off[s][*] = exclusive prefix of hist[s][*] over the workgroups, tot[s] = the slice's probes.
__global__ __launch_bounds__(256) void bloom_hist_scan_kernel(BloomPart p) {
  __shared__ uint32_t part[256 / 64];
  __shared__ uint32_t carry_s;
  const uint32_t* row = p.hist + (uint64_t)blockIdx.x * p.nwg;
  uint32_t* orow = p.off + (uint64_t)blockIdx.x * p.nwg;
  if (threadIdx.x == 0) carry_s = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  for (uint32_t b = 0; b < p.nwg; b += 256) {
    const uint32_t w = b + threadIdx.x;
    const uint32_t v = w < p.nwg ? row[w] : 0u;
    uint32_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)x, o);
      if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) part[wid] = x;
    __syncthreads();
    uint32_t before = carry_s;
    for (uint32_t q = 0; q < wid; q++) before += part[q];
    if (w < p.nwg) orow[w] = before + x - v;
    __syncthreads();
    if (threadIdx.x == 255) carry_s = before + x;
    __syncthreads();
  }
  if (threadIdx.x == 0) p.tot[blockIdx.x] = carry_s;
}

// base[s] = exclusive prefix of tot (one workgroup; S <= kBloomMaxSlices).
__global__ __launch_bounds__(1024) void bloom_base_scan_kernel(BloomPart p) {
  __shared__ uint32_t part[1024 / 64];
  __shared__ uint32_t carry_s;
  if (threadIdx.x == 0) carry_s = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  for (uint32_t b = 0; b < p.S; b += 1024) {
    const uint32_t s = b + threadIdx.x;
    const uint32_t v = s < p.S ? p.tot[s] : 0u;
    uint32_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)x, o);
      if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) part[wid] = x;
    __syncthreads();
    uint32_t before = carry_s;
    for (uint32_t q = 0; q < wid; q++) before += part[q];
    if (s < p.S) p.base[s] = before + x - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry_s = before + x;
    __syncthreads();
  }
}

// The workgroup's probes are placed in LDS grouped by slice (local offsets from its own counts),
// then written out in order: consecutive probes of one slice go to consecutive bucket slots, so
// the stores come out as runs instead of one scattered 4-byte store per probe.
__global__ __launch_bounds__(256) void bloom_scatter_kernel(BloomPart p) {
  extern __shared__ uint32_t lds[];
  uint32_t* loc = lds;                    // S: the local exclusive prefix (then the cursors)
  uint32_t* gof = lds + p.S;              // S: global slot of the slice's first local probe
  uint32_t* pr = lds + 2 * p.S;           // kBloomWgProbes: slice << 18 | bit in slice
  __shared__ uint32_t part[256 / 64];
  __shared__ uint32_t carry_s;
  if (threadIdx.x == 0) carry_s = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  for (uint32_t b = 0; b < p.S; b += 256) {       // block scan of this workgroup's counts
    const uint32_t sl = b + threadIdx.x;
    const uint64_t e = (uint64_t)sl * p.nwg + blockIdx.x;
    const uint32_t v = sl < p.S ? p.hist[e] : 0u;
    uint32_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)x, o);
      if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) part[wid] = x;
    __syncthreads();
    uint32_t before = carry_s;
    for (uint32_t q = 0; q < wid; q++) before += part[q];
    if (sl < p.S) {
      loc[sl] = before + x - v;
      gof[sl] = p.base[sl] + p.off[e];
    }
    __syncthreads();
    if (threadIdx.x == 255) carry_s = before + x;
    __syncthreads();
  }
  const uint32_t total = carry_s;
  const uint64_t i0 = (uint64_t)blockIdx.x * p.per_wg;
  const uint64_t i1 = min((uint64_t)p.n_keys, i0 + p.per_wg);
  for (uint64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const uint64_t s = p.key_pos[i];
    uint64_t h = xxh3::hash64(p.keys + s, p.key_pos[i + 1] - s);
    const uint64_t delta = (h >> 34) | (h << 30);   // Bloom::delta
    for (uint32_t j = 0; j < p.k; j++) {
      const uint64_t bit = h % p.limit;
      const uint32_t sl = (uint32_t)(bit >> kBloomSliceLog);
      const uint32_t r = atomicAdd(&loc[sl], 1u);   // LDS: loc[sl] ends at the next slice's start
      pr[r] = sl << kBloomSliceLog | (uint32_t)(bit & (kBloomSliceBits - 1));
      h += delta;
    }
  }
  __syncthreads();
  // loc[sl] is now the end of slice sl's local run; its start is loc[sl] - count
  for (uint32_t q = threadIdx.x; q < total; q += blockDim.x) {
    const uint32_t v = pr[q], sl = v >> kBloomSliceLog;
    const uint32_t start = loc[sl] - p.hist[(uint64_t)sl * p.nwg + blockIdx.x];
    p.pos[(uint64_t)gof[sl] + (q - start)] = v & (kBloomSliceBits - 1);
  }
}

// The gather path (TPZ_BLOOM_GATHER, a measured alternative: 1.66 ms against the scatter path's
// 1.24 ms for 35.6 M keys, the gathered ~38-probe runs being latency-bound): one pass over the keys. A workgroup counts its probes per slice,
// scans the counts (hist / off = its per-slice counts and local offsets, slice-major), hashes its
// keys again (L2-resident) to place the probes grouped by slice in LDS, and stores them as one
// contiguous block of its own. A workgroup per slice then gathers the slice's run from every
// workgroup's block (thread t takes runs t, t + 1024, ...; eight loads in flight per batch).
__global__ __launch_bounds__(256) void bloom_stage_kernel(BloomPart p) {
  extern __shared__ uint32_t lds[];
  uint32_t* cnt = lds;                    // S
  uint32_t* cur = lds + p.S;              // S
  uint32_t* pr = lds + 2 * p.S;           // kBloomWgProbes
  __shared__ uint32_t part[256 / 64];
  __shared__ uint32_t carry_s;
  for (uint32_t sl = threadIdx.x; sl < p.S; sl += blockDim.x) cnt[sl] = 0;
  if (threadIdx.x == 0) carry_s = 0;
  __syncthreads();
  bloom_count_pass(p, cnt);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  for (uint32_t b = 0; b < p.S; b += 256) {
    const uint32_t sl = b + threadIdx.x;
    const uint32_t v = sl < p.S ? cnt[sl] : 0u;
    uint32_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)x, o);
      if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) part[wid] = x;
    __syncthreads();
    uint32_t before = carry_s;
    for (uint32_t q = 0; q < wid; q++) before += part[q];
    if (sl < p.S) {
      cur[sl] = before + x - v;
      const uint64_t e = (uint64_t)sl * p.nwg + blockIdx.x;
      p.hist[e] = v;
      p.off[e] = before + x - v;
    }
    __syncthreads();
    if (threadIdx.x == 255) carry_s = before + x;
    __syncthreads();
  }
  const uint32_t total = carry_s;
  const uint64_t i0 = (uint64_t)blockIdx.x * p.per_wg;
  const uint64_t i1 = min((uint64_t)p.n_keys, i0 + p.per_wg);
  for (uint64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const uint64_t s = p.key_pos[i];
    uint64_t h = xxh3::hash64(p.keys + s, p.key_pos[i + 1] - s);
    const uint64_t delta = (h >> 34) | (h << 30);   // Bloom::delta
    for (uint32_t j = 0; j < p.k; j++) {
      const uint64_t bit = h % p.limit;
      const uint32_t r = atomicAdd(&cur[(uint32_t)(bit >> kBloomSliceLog)], 1u);   // LDS
      pr[r] = (uint32_t)(bit & (kBloomSliceBits - 1));
      h += delta;
    }
  }
  __syncthreads();
  uint32_t* dst = p.stage + (uint64_t)blockIdx.x * kBloomWgProbes;
  for (uint32_t q = threadIdx.x; q < total; q += blockDim.x) dst[q] = pr[q];
}

__global__ __launch_bounds__(1024) void bloom_gather_kernel(BloomPart p) {
  __shared__ uint32_t sl[kBloomSliceBits / 32];
  for (uint32_t w = threadIdx.x; w < kBloomSliceBits / 32; w += blockDim.x) sl[w] = 0;
  __syncthreads();
  const uint64_t row = (uint64_t)blockIdx.x * p.nwg;
  for (uint32_t w = threadIdx.x; w < p.nwg; w += blockDim.x) {
    const uint32_t c = p.hist[row + w], o = p.off[row + w];
    const uint32_t* src = p.stage + (uint64_t)w * kBloomWgProbes + o;
    for (uint32_t i = 0; i < c; i += 8) {
      uint32_t v[8];
#pragma unroll
      for (uint32_t r = 0; r < 8; r++) v[r] = i + r < c ? src[i + r] : 0u;
#pragma unroll
      for (uint32_t r = 0; r < 8; r++)
        if (i + r < c) atomicOr(&sl[v[r] >> 5], 1u << (v[r] & 31));   // LDS
    }
  }
  __syncthreads();
  const uint64_t w0 = (uint64_t)blockIdx.x * (kBloomSliceBits / 32);
  for (uint32_t w = threadIdx.x; w < kBloomSliceBits / 32; w += blockDim.x)
    if (w0 + w < p.filter_words) p.words[w0 + w] = sl[w];
}

// Slice s: OR its bucket into LDS, then store the slice's words (those below filter_words).
__global__ __launch_bounds__(1024) void bloom_fill_kernel(BloomPart p) {
  __shared__ uint32_t sl[kBloomSliceBits / 32];
  for (uint32_t w = threadIdx.x; w < kBloomSliceBits / 32; w += blockDim.x) sl[w] = 0;
  __syncthreads();
  const uint32_t b0 = p.base[blockIdx.x], n = p.tot[blockIdx.x];
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    const uint32_t b = p.pos[(uint64_t)b0 + i];
    atomicOr(&sl[b >> 5], 1u << (b & 31));          // LDS
  }
  __syncthreads();
  const uint64_t w0 = (uint64_t)blockIdx.x * (kBloomSliceBits / 32);
  for (uint32_t w = threadIdx.x; w < kBloomSliceBits / 32; w += blockDim.x)
    if (w0 + w < p.filter_words) p.words[w0 + w] = sl[w];
}

// Dense entry ends: block b's count[b] {kend, vend} pairs (status OK: from its worst-case-sized
// slot, tpz_entry_base; OK_SPILLED: from its spill record; zeros otherwise) moved to
// dense[2 * first[b] ..]. One wave per block.
__global__ __launch_bounds__(256) void pack_ends_kernel(PackLaunch a, uint2* dense) {
  const u32 lane = threadIdx.x & 63u;
  const u32 nw = gridDim.x * (blockDim.x >> 6);
  for (u32 b = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); b < a.n_blocks; b += nw) {
    const u64 f = a.first[b], c = a.first[b + 1] - f;
    const u32 st = a.status[b];
    const bool ok = block_decoded(st);
    const uint2* src = block_in_spill(st)
                           ? reinterpret_cast<const uint2*>(a.spill + a.spill_off[b])
                           : reinterpret_cast<const uint2*>(a.ends) + ends_base(a.efirst, a.ext[b], b);
    for (u64 j = lane; j < c; j += 64) dense[f + j] = ok ? src[j] : make_uint2(0, 0);
  }
}

// first[i] = sum of count[j] for j < i over the decoded blocks (OK / OK_SPILLED), i <= n: one
// 1024-thread workgroup, each thread a contiguous run (the host pipeline's chunks are <= 2^20).
__global__ __launch_bounds__(1024) void count_prefix_kernel(const u32* count, const uint8_t* status,
                                                            u32 n, u64* first) {
  __shared__ u64 part[1024];
  const u32 t = threadIdx.x, per = (n + 1023) / 1024;
  const u32 lo = min(n, t * per), hi = min(n, lo + per);
  u64 s = 0;
  for (u32 i = lo; i < hi; i++)
    s += block_decoded(status[i]) ? count[i] : 0u;
  part[t] = s;
  __syncthreads();
  for (u32 o = 1; o < 1024; o <<= 1) {          // Hillis-Steele inclusive scan of the parts
    const u64 v = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  u64 run = t ? part[t - 1] : 0;
  for (u32 i = lo; i < hi; i++) {
    first[i] = run;
    run += block_decoded(status[i]) ? count[i] : 0u;
  }
  if (t == 1023) first[n] = part[1023];
}

// The exact ends layout's reservation for block b: its header n when the decode parses it in
// place and writes its pairs to d_ends (uncompressed tag, len >= 7 + 2n: block.rs:49-59 pass;
// 6n <= len: the slot holds it), else 0 (tpz_gpu.h, tpz_entry_first).
__device__ __forceinline__ u32 exact_entries(const uint8_t* src, const u64* ext, u64 src_bytes,
                                             u32 b) {
  const u64 e0 = ext[b], e1 = ext[b + 1];
  if (e1 < e0 || e1 > src_bytes || e1 - e0 < 7) return 0;
  const u32 len = (u32)min(e1 - e0, (u64)0xffffffffu);
  if (src[e1 - 1] != 1) return 0;
  const u32 n = ((u32)src[e0] << 8) | src[e0 + 1];
  return (len >= 7 + 2 * n && 6 * n <= len) ? n : 0;
}

constexpr u32 kEfPer = 4;                 // blocks per thread
constexpr u32 kEfWg = 256 * kEfPer;       // blocks per workgroup

// Inclusive scan over the 256 threads of a workgroup (a shuffle prefix per wave, then
// the 4 wave totals).
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

__global__ __launch_bounds__(256) void entry_first_count(const uint8_t* src, const u64* ext,
                                                         u64 src_bytes, u32 n, u64* part) {
  __shared__ u64 wsum[4];
  const u64 b0 = (u64)blockIdx.x * kEfWg + threadIdx.x * kEfPer;
  u64 s = 0;
  for (u32 j = 0; j < kEfPer; j++)
    if (b0 + j < n) s += exact_entries(src, ext, src_bytes, (u32)(b0 + j));
  s = wg_inclusive(s, wsum);
  if (threadIdx.x == 255) part[blockIdx.x] = s;
}

// Exclusive scan of the workgroup totals in place, total at part[n_parts] (one workgroup).
__global__ __launch_bounds__(1024) void entry_first_parts_scan(u64* part, u32 n_parts) {
  __shared__ u64 acc[1024];
  const u32 t = threadIdx.x, per = (n_parts + 1023) / 1024;
  const u32 lo = min(n_parts, t * per), hi = min(n_parts, lo + per);
  u64 s = 0;
  for (u32 i = lo; i < hi; i++) s += part[i];
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
    const u64 x = part[i];
    part[i] = run;
    run += x;
  }
  if (t == 1023) part[n_parts] = acc[1023];
}

__global__ __launch_bounds__(256) void entry_first_write(const uint8_t* src, const u64* ext,
                                                         u64 src_bytes, u32 n, const u64* part,
                                                         u32 n_parts, u64* first) {
  __shared__ u64 wsum[4];
  const u64 b0 = (u64)blockIdx.x * kEfWg + threadIdx.x * kEfPer;
  u32 c[kEfPer];
  u64 s = 0;
  for (u32 j = 0; j < kEfPer; j++) {
    c[j] = b0 + j < n ? exact_entries(src, ext, src_bytes, (u32)(b0 + j)) : 0;
    s += c[j];
  }
  u64 run = wg_inclusive(s, wsum) - s + part[blockIdx.x];
  for (u32 j = 0; j < kEfPer; j++) {
    if (b0 + j < n) first[b0 + j] = run;
    run += c[j];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) first[n] = part[n_parts];
}

}  // namespace

uint64_t entry_first_parts(uint32_t n_blocks) { return (n_blocks + kEfWg - 1) / kEfWg + 1; }

void launch_entry_first(const uint8_t* src, const u64* ext, u64 src_bytes, u32 n_blocks,
                        u64* first, u64* part, hipStream_t stream) {
  if (n_blocks == 0) {
    (void)hipMemsetAsync(first, 0, 8, stream);
    return;
  }
  const u32 parts = (u32)entry_first_parts(n_blocks) - 1;
  hipLaunchKernelGGL(entry_first_count, dim3(parts), dim3(256), 0, stream, src, ext, src_bytes,
                     n_blocks, part);
  hipLaunchKernelGGL(entry_first_parts_scan, dim3(1), dim3(1024), 0, stream, part, parts);
  hipLaunchKernelGGL(entry_first_write, dim3(parts), dim3(256), 0, stream, src, ext, src_bytes,
                     n_blocks, part, parts, first);
}

void launch_count_prefix(const u32* count, const uint8_t* status, u32 n, u64* first,
                         hipStream_t stream) {
  hipLaunchKernelGGL(count_prefix_kernel, dim3(1), dim3(1024), 0, stream, count, status, n, first);
}

void launch_pack_ends(const PackLaunch& a, hipStream_t stream) {
  u32 grid = (a.n_blocks + 3) / 4;
  if (grid > 65535) grid = 65535;
  hipLaunchKernelGGL(pack_ends_kernel, dim3(grid), dim3(256), 0, stream, a,
                     reinterpret_cast<uint2*>(a.dense));
}

void launch_seek(const SeekLaunch& a, hipStream_t stream) {
  SeekParams p{a.fk, a.fk_pos, a.n_blocks, a.ext, a.data, a.ends, a.count, a.bstatus,
               a.spill, a.spill_off, a.q, a.q_pos, a.n_q, a.out_block, a.out_entry,
               a.out_status, a.out_valid, a.efirst};
  hipLaunchKernelGGL(seek_kernel, dim3((a.n_q + 255) / 256), dim3(256), 0, stream, p);
}

uint64_t bloom_build_work_bytes(uint32_t n_keys, uint32_t k, uint64_t limit) {
  const uint64_t S = (limit + kBloomSliceBits - 1) >> kBloomSliceLog;
  if (S == 0 || S > kBloomMaxSlices || (uint64_t)n_keys * k >= (1ull << 32)) return 0;
  const uint64_t nwg = bloom_part_wgs(n_keys, k);
  return 4ull * (nwg * kBloomWgProbes + 2 * S * nwg + 2 * S + 64);   // >= n_keys * k probes
}

void launch_bloom_build(const BloomBuildLaunch& a, hipStream_t stream) {
  if (!a.n_keys || !a.limit) return;
  const uint64_t S = (a.limit + kBloomSliceBits - 1) >> kBloomSliceLog;
  if (!a.work || S > kBloomMaxSlices) {
    hipLaunchKernelGGL(bloom_build_kernel, dim3((a.n_keys + 255) / 256), dim3(256), 0, stream, a);
    return;
  }
  BloomPart p{};
  p.keys = a.keys;
  p.key_pos = a.key_pos;
  p.n_keys = a.n_keys;
  p.k = a.k;
  p.limit = a.limit;
  p.S = (uint32_t)S;
  p.nwg = bloom_part_wgs(a.n_keys, a.k);
  p.per_wg = bloom_part_per_wg(a.k);
  uint32_t* w = static_cast<uint32_t*>(a.work);
  p.hist = w;                                    // S x nwg, slice-major
  p.off = w + (uint64_t)p.S * p.nwg;             // S x nwg
  p.tot = p.off + (uint64_t)p.S * p.nwg;         // S slice totals
  p.base = p.tot + p.S;                          // S slice bases
  p.pos = p.base + p.S + 64;                     // n_keys x k in-slice bit offsets
  p.stage = p.pos;                               // or nwg x kBloomWgProbes (gather path)
  p.words = reinterpret_cast<uint32_t*>(a.filter);
  p.filter_words = a.filter_words;
  static const bool gather = std::getenv("TPZ_BLOOM_GATHER") != nullptr;   // A/B probe
  if (gather) {
    hipLaunchKernelGGL(bloom_stage_kernel, dim3(p.nwg), dim3(256), (2 * p.S + kBloomWgProbes) * 4,
                       stream, p);
    hipLaunchKernelGGL(bloom_gather_kernel, dim3(p.S), dim3(1024), 0, stream, p);
    return;
  }
  hipLaunchKernelGGL(bloom_count_kernel, dim3(p.nwg), dim3(256), p.S * 4, stream, p);
  hipLaunchKernelGGL(bloom_hist_scan_kernel, dim3(p.S), dim3(256), 0, stream, p);
  hipLaunchKernelGGL(bloom_base_scan_kernel, dim3(1), dim3(1024), 0, stream, p);
  hipLaunchKernelGGL(bloom_scatter_kernel, dim3(p.nwg), dim3(256), (2 * p.S + kBloomWgProbes) * 4,
                     stream, p);
  hipLaunchKernelGGL(bloom_fill_kernel, dim3(p.S), dim3(1024), 0, stream, p);
}

void launch_bloom(const BloomLaunch& a, hipStream_t stream) {
  BloomParams p{a.filter, a.filter_len, a.q, a.q_pos, a.n_q, a.out};
  hipLaunchKernelGGL(bloom_kernel, dim3((a.n_q + 255) / 256), dim3(256), 0, stream, p);
}

}  // namespace tpz
