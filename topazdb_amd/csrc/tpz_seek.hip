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
// its panic for MALFORMED); OK_SPILLED blocks are read from their spill records and report OK.

#include <hip/hip_runtime.h>
#include <stdint.h>

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
};

// A decoded block's ends and stream: its slot, or its spill record (include/tpz_gpu.h).
struct BlockView {
  const u32* ends;
  const uint8_t* stream;
};
__device__ __forceinline__ BlockView block_view(const SeekParams& p, u32 b, u32 st) {
  if (st == TPZ_BLOCK_OK_SPILLED) {
    const uint8_t* r = p.spill + p.spill_off[b];
    return BlockView{reinterpret_cast<const u32*>(r), r + spill_stream(p.count[b])};
  }
  const u64 e0 = p.ext[b];
  return BlockView{p.ends + 2 * entry_base(e0, b), p.data + slot_base(e0, b)};
}
// Entry j's key: its bytes and length.
__device__ __forceinline__ const uint8_t* entry_key(const BlockView& v, u32 j, u64& len) {
  const u32 lo = j ? v.ends[2 * (j - 1)] : 0u, hi = v.ends[2 * j];
  len = hi - lo;
  return v.stream + lo;
}
__device__ __forceinline__ bool decoded(u32 st) {
  return st == TPZ_BLOCK_OK || st == TPZ_BLOCK_OK_SPILLED;
}

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
  bool valid = false;
  if (decoded(st)) {
    // BlockIterator::seek_to_key
    const BlockView v = block_view(p, b, st);
    const u32 n = p.count[b];
    u32 l = 0, r = n;
    pos = n;
    bool found = false;
    while (l < r) {
      const u32 mid = (r - l) / 2 + l;
      u64 kl;
      const uint8_t* k = entry_key(v, mid, kl);
      const int c = key_cmp(k, kl, qk, ql);
      if (c > 0) r = mid;
      else if (c < 0) l = mid + 1;
      else { pos = mid; found = true; break; }
    }
    if (!found) pos = l;
    u64 kl = 0;
    if (pos < n) entry_key(v, pos, kl);
    valid = pos < n && kl > 0;                // is_valid: the current key is non-empty
    if (!valid && b + 1 < p.n_blocks) {       // the next block, from its first entry
      b++;
      st = p.bstatus[b];
      pos = 0;
      valid = false;
      if (decoded(st) && p.count[b] > 0) {
        entry_key(block_view(p, b, st), 0, kl);
        valid = kl > 0;
      }
    }
  }
  p.out_block[i] = b;
  p.out_entry[i] = pos;
  p.out_status[i] = decoded(st) ? (uint8_t)TPZ_BLOCK_OK : (uint8_t)st;
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
    atomicOr(&words[bit >> 5], 1u << (bit & 31));           // bit_set: byte bit/8, bit bit%8
    h += delta;
  }
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
    const bool ok = st == TPZ_BLOCK_OK || st == TPZ_BLOCK_OK_SPILLED;
    const uint2* src = st == TPZ_BLOCK_OK_SPILLED
                           ? reinterpret_cast<const uint2*>(a.spill + a.spill_off[b])
                           : reinterpret_cast<const uint2*>(a.ends) + entry_base(a.ext[b], b);
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
    s += (status[i] == TPZ_BLOCK_OK || status[i] == TPZ_BLOCK_OK_SPILLED) ? count[i] : 0u;
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
    run += (status[i] == TPZ_BLOCK_OK || status[i] == TPZ_BLOCK_OK_SPILLED) ? count[i] : 0u;
  }
  if (t == 1023) first[n] = part[1023];
}

}  // namespace

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
               a.out_status, a.out_valid};
  hipLaunchKernelGGL(seek_kernel, dim3((a.n_q + 255) / 256), dim3(256), 0, stream, p);
}

void launch_bloom_build(const BloomBuildLaunch& a, hipStream_t stream) {
  if (a.n_keys && a.limit)
    hipLaunchKernelGGL(bloom_build_kernel, dim3((a.n_keys + 255) / 256), dim3(256), 0, stream, a);
}

void launch_bloom(const BloomLaunch& a, hipStream_t stream) {
  BloomParams p{a.filter, a.filter_len, a.q, a.q_pos, a.n_q, a.out};
  hipLaunchKernelGGL(bloom_kernel, dim3((a.n_q + 255) / 256), dim3(256), 0, stream, p);
}

}  // namespace tpz
