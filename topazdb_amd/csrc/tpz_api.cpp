// tpz_api.cpp — the C ABI of include/tpz_gpu.h: context, workspace, launches, error text.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "tpz_internal.h"
#include "tpz_xxh3.h"

namespace {

thread_local std::string g_last_error;

tpz_err hip_fail(hipError_t e, const char* what) {
  g_last_error = std::string(what) + ": " + hipGetErrorString(e);
  return TPZ_ERR_HIP;
}

#define TPZ_HIP(call)                                     \
  do {                                                    \
    hipError_t e_ = (call);                               \
    if (e_ != hipSuccess) return hip_fail(e_, #call);     \
  } while (0)

// T_k[b] = raw CRC-32 (reflected 0xEDB88320, init 0, no xorout) of byte b followed by k zero
// bytes; T_{k+1}[b] = (T_k[b] >> 8) ^ T_0[T_k[b] & 0xFF]. Only the 40 tables the kernels use
// are kept, plus the inverse of T_0's top byte (ids documented in tpz_internal.h).
std::vector<uint32_t> build_crc_tables() {
  const int kmax = 5120;
  std::vector<uint32_t> all((size_t)kmax * 256);
  for (uint32_t b = 0; b < 256; b++) {
    uint32_t c = b;
    for (int i = 0; i < 8; i++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    all[b] = c;
  }
  for (int k = 1; k < kmax; k++)
    for (uint32_t b = 0; b < 256; b++) {
      uint32_t t = all[(size_t)(k - 1) * 256 + b];
      all[(size_t)k * 256 + b] = (t >> 8) ^ all[t & 0xFF];
    }
  std::vector<uint32_t> out((size_t)tpz::kNumCrcTables * 256);
  auto put = [&](int id, int k) {
    std::memcpy(&out[(size_t)id * 256], &all[(size_t)k * 256], 256 * 4);
  };
  for (int k = 0; k < 16; k++) put(k, k);
  for (int j = 0; j < 6; j++) {
    const int n = tpz::kCrcShiftBytes[j];
    for (int i = 0; i < 4; i++) put(16 + 4 * j + i, n - 1 - i);
  }
  for (uint32_t b = 0; b < 256; b++) out[(size_t)tpz::kCrcInvTable * 256 + (all[b] >> 24)] = b;
  return out;
}

// GF(2) polynomials modulo the reflected CRC-32 polynomial, bit 31 = x^0 (zlib's crc32.c
// multmodp / x2nmodp, restated): a * b mod P, for a != 0.
uint32_t multmodp(uint32_t a, uint32_t b) {
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = (b & 1) ? (b >> 1) ^ 0xEDB88320u : b >> 1;
  }
  return p;
}
// x^(8n) mod P: the operator "append n zero bytes" (Z_n(a) = multmodp(x8n(n), a)).
uint32_t x8n(uint64_t n) {
  uint32_t x2k[64];
  x2k[0] = 1u << 30;  // x^1
  for (int k = 1; k < 64; k++) x2k[k] = multmodp(x2k[k - 1], x2k[k - 1]);  // x^(2^k)
  uint32_t p = 1u << 31;  // x^0
  for (int k = 3; n; n >>= 1, k++)
    if (n & 1) p = multmodp(x2k[k], p);
  return p;
}

// Range-CRC tables (tpz_crc.hip): ids 0..15 = T_0..T_15; ids 16 + 4j + i = T_{n-1-i},
// n = 16 * 2^j; T_k[b] = Z_k(T_0[b]).
std::vector<uint32_t> build_range_tables() {
  uint32_t t0[256];
  for (uint32_t b = 0; b < 256; b++) {
    uint32_t c = b;
    for (int i = 0; i < 8; i++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    t0[b] = c;
  }
  std::vector<uint32_t> out((size_t)tpz::kRangeTablesAll * 256);
  auto put = [&](int id, uint64_t k) {
    const uint32_t z = x8n(k);
    for (uint32_t b = 0; b < 256; b++) out[(size_t)id * 256 + b] = t0[b] ? multmodp(z, t0[b]) : 0u;
  };
  for (int k = 0; k < 16; k++) put(k, (uint64_t)k);
  for (int j = 0; j < tpz::kRangeShiftOps; j++) {
    const uint64_t n = 16ull << j;
    for (int i = 0; i < 4; i++) put(16 + 4 * j + i, n - 1 - (uint64_t)i);
  }
  for (int i = 0; i < 4; i++)
    for (uint64_t j = 0; j < 256; j++)
      out[(size_t)(tpz::kPowTable + i) * 256 + j] = x8n(j << (8 * i));
  return out;
}

// The slice-by-4 tables T_0..T_3 replicated 32 times: word (t*256 + b)*32 + r = T_t[b].
std::vector<uint32_t> build_rep_tables(const std::vector<uint32_t>& range) {
  std::vector<uint32_t> out((size_t)tpz::kCrcRepWords);
  for (int t = 0; t < 4; t++)
    for (int b = 0; b < 256; b++)
      for (int r = 0; r < 32; r++) out[((size_t)t * 256 + b) * 32 + r] = range[(size_t)t * 256 + b];
  return out;
}

}  // namespace

// Device workspace of one stream: the big-path and spill-path worklists, the big path's
// per-workgroup entry tables and the range-CRC accumulators. Decodes on different streams run
// concurrently, so each stream has its own; calls on one stream are ordered by the stream.
struct tpz_workspace {
  uint32_t* d_defer = nullptr;  // [0] big/codec counter, [1] spill counter, [2] bigwave counter,
                                // [4, 4 + cap) big or codec list, [4 + cap, 4 + 2 cap) spill list,
                                // [4 + 2 cap, 4 + 3 cap) bigwave list
  uint32_t defer_cap = 0;
  uint32_t* d_tail = nullptr;   // the decode's tpz::kTailCounters (zero between decodes) + the
                                // sticky tpz::kTailError word
  uint64_t* d_big_scratch = nullptr;
  uint32_t* d_acc = nullptr;    // acc_cap per-range accumulators of tpz_crc32_ranges
  uint32_t acc_cap = 0;
  void* d_plan0 = nullptr;      // tpz_plan_blocks: nx + per-workgroup maxima + info
  size_t plan0_cap = 0;
  void* d_plan1 = nullptr;      // tpz_plan_blocks: the transfer tables + chunk counts
  size_t plan1_cap = 0;
  void* d_bloom = nullptr;      // tpz_bloom_build: probe buckets + slice histograms
  size_t bloom_cap = 0;
  void* d_comp = nullptr;       // tpz_compress_blocks: the per-block scratch slots + scan parts
  size_t comp_cap = 0;
  uint32_t* h_info = nullptr;   // pinned: tpz_plan_blocks' read-back of its 16-byte info
};

struct tpz_ctx {
  int device = 0;
  uint32_t num_cus = 0;
  uint32_t* d_tables = nullptr;        // block-decode CRC tables
  uint32_t* d_range_tables = nullptr;  // range-CRC tables
  uint32_t* d_rep_tables = nullptr;    // replicated slice-by-4 tables
  std::mutex mu;  // guards the workspace map and the host pipelines
  std::unordered_map<void*, tpz_workspace> ws;
  std::vector<void*> pipes;        // every host pipeline of the context (owned)
  std::vector<void*> pipes_free;   // those not in use by a tpz_decode_blocks_host call
};

namespace {

void free_workspace(tpz_workspace& w) {
  if (w.d_defer) (void)hipFree(w.d_defer);
  if (w.d_tail) (void)hipFree(w.d_tail);
  if (w.d_big_scratch) (void)hipFree(w.d_big_scratch);
  if (w.d_acc) (void)hipFree(w.d_acc);
  if (w.d_plan0) (void)hipFree(w.d_plan0);
  if (w.d_plan1) (void)hipFree(w.d_plan1);
  if (w.d_bloom) (void)hipFree(w.d_bloom);
  if (w.d_comp) (void)hipFree(w.d_comp);
  if (w.h_info) (void)hipHostFree(w.h_info);
  w = tpz_workspace{};
}

// The stream's range-CRC accumulators, grown to n ranges. Caller holds c->mu.
tpz_err get_acc(tpz_ctx* c, void* stream, uint32_t n, uint32_t** out) {
  tpz_workspace& w = c->ws[stream];
  if (!w.d_acc || w.acc_cap < n) {
    uint32_t* d = nullptr;
    TPZ_HIP(hipMalloc(&d, (size_t)n * 4));
    if (w.d_acc) {
      (void)hipStreamSynchronize((hipStream_t)stream);
      (void)hipFree(w.d_acc);
    }
    w.d_acc = d;
    w.acc_cap = n;
  }
  *out = w.d_acc;
  return TPZ_SUCCESS;
}

// A grow-only device buffer of the stream's workspace (the stream is idle or only uses it in
// order: a buffer is replaced after the stream's pending work is done). Caller holds c->mu.
tpz_err grow(void* stream, void** buf, size_t* cap, size_t bytes) {
  if (*buf && *cap >= bytes) return TPZ_SUCCESS;
  void* d = nullptr;
  TPZ_HIP(hipMalloc(&d, bytes));
  if (*buf) {
    (void)hipStreamSynchronize((hipStream_t)stream);
    (void)hipFree(*buf);
  }
  *buf = d;
  *cap = bytes;
  return TPZ_SUCCESS;
}

// The stream's workspace, grown to max_blocks. Caller holds c->mu.
tpz_err get_workspace(tpz_ctx* c, void* stream, uint32_t max_blocks, tpz_workspace** out) {
  tpz_workspace& w = c->ws[stream];
  if (!w.d_big_scratch)
    TPZ_HIP(hipMalloc(&w.d_big_scratch, (size_t)c->num_cus * 2 * tpz::kBigMaxSlots * sizeof(uint64_t)));
  if (!w.d_tail) {
    TPZ_HIP(hipMalloc(&w.d_tail, tpz::kTailWords * sizeof(uint32_t)));
    TPZ_HIP(hipMemsetAsync(w.d_tail, 0, tpz::kTailWords * sizeof(uint32_t), (hipStream_t)stream));
  }
  if (!w.d_defer || w.defer_cap < max_blocks) {
    uint32_t* d = nullptr;
    TPZ_HIP(hipMalloc(&d, (3 * (size_t)max_blocks + 4) * 4));
    if (w.d_defer) {
      // an earlier decode on this stream may still be reading the old list
      (void)hipStreamSynchronize((hipStream_t)stream);
      (void)hipFree(w.d_defer);
    }
    w.d_defer = d;
    w.defer_cap = max_blocks;
  }
  *out = &w;
  return TPZ_SUCCESS;
}

}  // namespace

int tpz_internal_device(tpz_ctx* c) { return c->device; }
void* tpz_internal_pipe_acquire(tpz_ctx* c) {
  std::lock_guard<std::mutex> g(c->mu);
  if (c->pipes_free.empty()) return nullptr;
  void* p = c->pipes_free.back();
  c->pipes_free.pop_back();
  return p;
}
void tpz_internal_pipe_release(tpz_ctx* c, void* pipe, bool fresh) {
  std::lock_guard<std::mutex> g(c->mu);
  if (fresh) c->pipes.push_back(pipe);
  c->pipes_free.push_back(pipe);
}
tpz_err tpz_internal_hip_fail(hipError_t e, const char* what) { return hip_fail(e, what); }
tpz_err tpz_internal_fail(tpz_err err, const char* what) {
  g_last_error = what;
  return err;
}

extern "C" {

uint64_t tpz_layout_slot_base(uint64_t ext_i, uint64_t i) { return tpz_slot_base(ext_i, i); }
uint64_t tpz_layout_value_start(uint64_t key_bytes) { return tpz_value_start(key_bytes); }
uint64_t tpz_layout_entry_base(uint64_t ext_i, uint64_t i) { return tpz_entry_base(ext_i, i); }
uint64_t tpz_layout_data_capacity(uint64_t s, uint64_t n) { return tpz_data_capacity(s, n); }
uint64_t tpz_layout_entry_capacity(uint64_t s, uint64_t n) { return tpz_entry_capacity(s, n); }
uint64_t tpz_layout_spill_stream(uint64_t n) { return tpz_spill_stream(n); }
uint64_t tpz_layout_spill_classes(uint64_t n, uint64_t k, uint64_t v) {
  return tpz_spill_classes(n, k, v);
}
int tpz_abi_version(void) { return TPZ_ABI_VERSION; }

const char* tpz_last_error(void) { return g_last_error.c_str(); }

tpz_err tpz_ctx_create(int device, tpz_ctx** out) {
  if (!out) return TPZ_ERR_INVALID_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
    g_last_error = "no HIP device " + std::to_string(device);
    return TPZ_ERR_NO_DEVICE;
  }
  hipDeviceProp_t prop;
  TPZ_HIP(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    g_last_error = std::string("device is ") + prop.gcnArchName + ", kernels are built for gfx950";
    return TPZ_ERR_NO_DEVICE;
  }
  TPZ_HIP(hipSetDevice(device));
  tpz_ctx* c = new tpz_ctx();
  c->device = device;
  c->num_cus = (uint32_t)prop.multiProcessorCount;
  const std::vector<uint32_t> t = build_crc_tables();
  const std::vector<uint32_t> rt = build_range_tables();
  const std::vector<uint32_t> rep = build_rep_tables(rt);
  hipError_t e = hipSuccess;
  for (auto [dst, v] : {std::make_pair(&c->d_tables, &t), std::make_pair(&c->d_range_tables, &rt),
                        std::make_pair(&c->d_rep_tables, &rep)}) {
    if (e == hipSuccess) e = hipMalloc(dst, v->size() * 4);
    if (e == hipSuccess) e = hipMemcpy(*dst, v->data(), v->size() * 4, hipMemcpyHostToDevice);
  }
  if (e != hipSuccess) {
    tpz_ctx_destroy(c);
    return hip_fail(e, "tpz_ctx_create");
  }
  *out = c;
  return TPZ_SUCCESS;
}

void tpz_ctx_destroy(tpz_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipDeviceSynchronize();  // decodes still in flight use the workspaces
  if (c->d_tables) (void)hipFree(c->d_tables);
  if (c->d_range_tables) (void)hipFree(c->d_range_tables);
  if (c->d_rep_tables) (void)hipFree(c->d_rep_tables);
  for (auto& kv : c->ws) free_workspace(kv.second);
  for (void* p : c->pipes) tpz_internal_pipe_destroy(p);
  delete c;
}

tpz_err tpz_ctx_reserve(tpz_ctx* c, uint32_t max_blocks, void* stream) {
  if (!c) return TPZ_ERR_INVALID_ARG;
  TPZ_HIP(hipSetDevice(c->device));
  std::lock_guard<std::mutex> g(c->mu);
  tpz_workspace* w = nullptr;
  return get_workspace(c, stream, max_blocks, &w);
}

tpz_err tpz_decode_blocks(tpz_ctx* c, const tpz_batch* b, const tpz_columns* o, void* stream) {
  if (!c || !b || !o) return TPZ_ERR_INVALID_ARG;
  if (b->n_blocks == 0) {
    if (o->d_spill_used) {
      TPZ_HIP(hipSetDevice(c->device));
      TPZ_HIP(hipMemsetAsync(o->d_spill_used, 0, 8, (hipStream_t)stream));
    }
    return TPZ_SUCCESS;
  }
  if (!b->d_src || !b->d_ext || !o->d_data || !o->d_ends || !o->d_count || !o->d_status ||
      !o->d_crc || !o->d_spill_off || !o->d_spill_used || (o->spill_cap && !o->d_spill) ||
      (reinterpret_cast<uintptr_t>(b->d_src) & 15u))
    return TPZ_ERR_INVALID_ARG;
  TPZ_HIP(hipSetDevice(c->device));
  tpz_workspace* w = nullptr;
  {
    std::lock_guard<std::mutex> g(c->mu);
    tpz_err r = get_workspace(c, stream, b->n_blocks, &w);
    if (r != TPZ_SUCCESS) return r;
  }
  uint32_t* tail = w->d_tail;
  hipStream_t s = (hipStream_t)stream;
  tpz::LaunchArgs a{};
  a.src = b->d_src;
  a.ext = b->d_ext;
  a.src_bytes = b->src_bytes;
  a.n_blocks = b->n_blocks;
  a.crc_tables = c->d_tables;
  a.data = o->d_data;
  a.ends = o->d_ends;
  a.count = o->d_count;
  a.status = o->d_status;
  a.crc = o->d_crc;
  a.tail = tail;
  a.defer_count = tail + tpz::kTailBig;
  a.defer_list = w->d_defer + 4;
  a.spill_count = tail + tpz::kTailSpill;
  a.spill_list = w->d_defer + 4 + w->defer_cap;
  a.bw_count = tail + tpz::kTailBw;
  a.bw_list = w->d_defer + 4 + 2 * (size_t)w->defer_cap;
  a.rep = c->d_rep_tables;
  a.spill = o->d_spill;
  a.spill_cap = o->d_spill ? o->spill_cap : 0;
  a.spill_off = o->d_spill_off;
  a.spill_used = o->d_spill_used;   // zeroed by the first kernel
  a.num_cus = c->num_cus;
  a.big_scratch = w->d_big_scratch;
  a.big_grid = c->num_cus;
  a.efirst = o->d_entry_first;
  tpz::launch_decode(a, s);
  TPZ_HIP(hipGetLastError());
  return TPZ_SUCCESS;
}

tpz_err tpz_decode_check(tpz_ctx* c, void* stream) {
  if (!c) return TPZ_ERR_INVALID_ARG;
  TPZ_HIP(hipSetDevice(c->device));
  uint32_t* tail = nullptr;
  {
    std::lock_guard<std::mutex> g(c->mu);
    auto it = c->ws.find(stream);
    if (it != c->ws.end()) tail = it->second.d_tail;
  }
  hipStream_t s = (hipStream_t)stream;
  if (!tail) return hip_fail(hipStreamSynchronize(s), "tpz_decode_check");
  // read and clear the stream's flag in stream order (after every decode queued before it; the
  // null stream is not involved), then wait for both
  uint32_t flag = 0;
  TPZ_HIP(hipMemcpyAsync(&flag, tail + tpz::kTailError, 4, hipMemcpyDeviceToHost, s));
  TPZ_HIP(hipMemsetAsync(tail + tpz::kTailError, 0, 4, s));
  TPZ_HIP(hipStreamSynchronize(s));
  if (!flag) return TPZ_SUCCESS;
  // bit 0: a tail workgroup's bounded wait; bit 1: a wave path row wait; bit 2: a wave path row
  // slot overwritten before its reader got to it (tpz_decode.hip claim_chunk)
  g_last_error = (flag & 1u) ? "tpz_decode_blocks: a tail workgroup's wait for the big path timed out; "
                               "spill blocks of a batch on this stream may be undecoded"
                             : "tpz_decode_blocks: a wave path row claim timed out or was overwritten; "
                               "blocks of a batch on this stream may be undecoded";
  return TPZ_ERR_INTERNAL;
}

static tpz_err crc_ranges(tpz_ctx* c, const tpz_batch* r, uint32_t trailer, uint32_t* d_crc,
                          uint8_t* d_status, void* stream) {
  if (!c || !r || !d_crc) return TPZ_ERR_INVALID_ARG;
  if (r->n_blocks == 0) return TPZ_SUCCESS;
  if (!r->d_src || !r->d_ext) return TPZ_ERR_INVALID_ARG;
  TPZ_HIP(hipSetDevice(c->device));
  uint32_t* acc = nullptr;
  {
    std::lock_guard<std::mutex> g(c->mu);
    tpz_err e = get_acc(c, stream, r->n_blocks, &acc);
    if (e != TPZ_SUCCESS) return e;
  }
  hipStream_t s = (hipStream_t)stream;
  TPZ_HIP(hipMemsetAsync(acc, 0, (size_t)r->n_blocks * 4, s));
  tpz::CrcLaunch a{};
  a.src = r->d_src;
  a.ext = r->d_ext;
  a.src_bytes = r->src_bytes;
  a.n_ranges = r->n_blocks;
  a.trailer = trailer;
  a.tables = c->d_range_tables;
  a.rep = c->d_rep_tables;
  a.acc = acc;
  a.crc = d_crc;
  a.status = d_status;
  a.num_cus = c->num_cus;
  tpz::launch_crc_ranges(a, s);
  TPZ_HIP(hipGetLastError());
  return TPZ_SUCCESS;
}

static tpz_err decompressed_sizes(tpz_ctx* c, const tpz_batch* b, uint64_t* d_size, void* stream,
                                  bool claimed) {
  if (!c || !b || !d_size) return TPZ_ERR_INVALID_ARG;
  if (b->n_blocks == 0) return TPZ_SUCCESS;
  if (!b->d_src || !b->d_ext || (reinterpret_cast<uintptr_t>(b->d_src) & 15u))
    return TPZ_ERR_INVALID_ARG;
  TPZ_HIP(hipSetDevice(c->device));
  tpz::CodecLaunch a{};
  a.src = b->d_src;
  a.ext = b->d_ext;
  a.src_bytes = b->src_bytes;
  a.n_blocks = b->n_blocks;
  a.size = d_size;
  a.claimed = claimed;
  tpz::launch_codec_sizes(a, (hipStream_t)stream);
  TPZ_HIP(hipGetLastError());
  return TPZ_SUCCESS;
}

tpz_err tpz_decompressed_sizes(tpz_ctx* c, const tpz_batch* b, uint64_t* d_size, void* stream) {
  return decompressed_sizes(c, b, d_size, stream, false);
}

tpz_err tpz_decompressed_sizes_claimed(tpz_ctx* c, const tpz_batch* b, uint64_t* d_size,
                                       void* stream) {
  return decompressed_sizes(c, b, d_size, stream, true);
}

tpz_err tpz_decompress_check(tpz_ctx* c, void* stream) {
  if (!c) return TPZ_ERR_INVALID_ARG;
  TPZ_HIP(hipSetDevice(c->device));
  uint32_t* tail = nullptr;
  {
    std::lock_guard<std::mutex> g(c->mu);
    auto it = c->ws.find(stream);
    if (it != c->ws.end()) tail = it->second.d_tail;
  }
  hipStream_t s = (hipStream_t)stream;
  if (!tail) return hip_fail(hipStreamSynchronize(s), "tpz_decompress_check");
  // read and clear the stream's word in stream order, as tpz_decode_check does
  uint32_t flag = 0;
  TPZ_HIP(hipMemcpyAsync(&flag, tail + tpz::kTailCodecInexact, 4, hipMemcpyDeviceToHost, s));
  TPZ_HIP(hipMemsetAsync(tail + tpz::kTailCodecInexact, 0, 4, s));
  TPZ_HIP(hipStreamSynchronize(s));
  if (!flag) return TPZ_SUCCESS;
  g_last_error = "tpz_decompress_blocks: an LZ4 block's claimed size was not its decoded length "
                 "(an Err or a short stream); size the batch with tpz_decompressed_sizes and "
                 "decompress it again";
  return TPZ_ERR_SIZES;
}

tpz_err tpz_decompress_blocks(tpz_ctx* c, const tpz_batch* b, uint8_t* d_dst,
                              const uint64_t* d_dst_ext, uint8_t* d_status, void* stream) {
  if (!c || !b || !d_dst || !d_dst_ext || !d_status) return TPZ_ERR_INVALID_ARG;
  if (b->n_blocks == 0) return TPZ_SUCCESS;
  if (!b->d_src || !b->d_ext || (reinterpret_cast<uintptr_t>(b->d_src) & 15u))
    return TPZ_ERR_INVALID_ARG;
  TPZ_HIP(hipSetDevice(c->device));
  tpz_workspace* w = nullptr;
  {
    std::lock_guard<std::mutex> g(c->mu);
    tpz_err r = get_workspace(c, stream, b->n_blocks, &w);
    if (r != TPZ_SUCCESS) return r;
  }
  hipStream_t s = (hipStream_t)stream;
  tpz::CodecLaunch a{};
  a.src = b->d_src;
  a.ext = b->d_ext;
  a.src_bytes = b->src_bytes;
  a.n_blocks = b->n_blocks;
  a.dst = d_dst;
  a.dst_ext = d_dst_ext;
  a.status = d_status;
  a.defer_count = w->d_defer;
  a.defer_list = w->d_defer + 4;
  a.num_cus = c->num_cus;
  a.inexact = w->d_tail + tpz::kTailCodecInexact;
  tpz::launch_decompress(a, s);
  TPZ_HIP(hipGetLastError());
  return TPZ_SUCCESS;
}

tpz_err tpz_entry_first(tpz_ctx* c, const tpz_batch* b, uint64_t* d_first, void* stream) {
  if (!c || !b || !d_first) return TPZ_ERR_INVALID_ARG;
  if (b->n_blocks && (!b->d_src || !b->d_ext)) return TPZ_ERR_INVALID_ARG;
  TPZ_HIP(hipSetDevice(c->device));
  uint32_t* part = nullptr;
  {
    std::lock_guard<std::mutex> g(c->mu);
    tpz_err e = get_acc(c, stream, 2 * (uint32_t)tpz::entry_first_parts(b->n_blocks), &part);
    if (e != TPZ_SUCCESS) return e;
  }
  tpz::launch_entry_first(b->d_src, b->d_ext, b->src_bytes, b->n_blocks, d_first,
                          reinterpret_cast<uint64_t*>(part), (hipStream_t)stream);
  TPZ_HIP(hipGetLastError());
  return TPZ_SUCCESS;
}

tpz_err tpz_flat_layout(tpz_ctx* c, const tpz_batch* b, uint64_t* d_first, void* stream) {
  if (!c || !b || !d_first) return TPZ_ERR_INVALID_ARG;
  if (b->n_blocks && (!b->d_src || !b->d_ext)) return TPZ_ERR_INVALID_ARG;
  TPZ_HIP(hipSetDevice(c->device));
  uint32_t* part = nullptr;
  {
    std::lock_guard<std::mutex> g(c->mu);
    tpz_err e = get_acc(c, stream, 2 * (uint32_t)tpz::flat_scan_parts_words(b->n_blocks), &part);
    if (e != TPZ_SUCCESS) return e;
  }
  tpz::launch_flat_layout(b->d_src, b->d_ext, b->src_bytes, b->n_blocks, d_first,
                          reinterpret_cast<uint64_t*>(part), c->num_cus, (hipStream_t)stream);
  TPZ_HIP(hipGetLastError());
  return TPZ_SUCCESS;
}

tpz_err tpz_decode_blocks_flat(tpz_ctx* c, const tpz_batch* b, const tpz_flat_columns* o,
                               void* stream) {
  if (!c || !b || !o) return TPZ_ERR_INVALID_ARG;
  if (b->n_blocks == 0) {
    if (o->d_spill_used) {
      TPZ_HIP(hipSetDevice(c->device));
      TPZ_HIP(hipMemsetAsync(o->d_spill_used, 0, 8, (hipStream_t)stream));
    }
    return TPZ_SUCCESS;
  }
  if (!b->d_src || !b->d_ext || !o->d_keys || !o->d_values || !o->d_ends || !o->d_first ||
      !o->d_count || !o->d_status || !o->d_crc || !o->d_spill_off || !o->d_spill_used ||
      (o->spill_cap && !o->d_spill) || (reinterpret_cast<uintptr_t>(b->d_src) & 15u) ||
      (reinterpret_cast<uintptr_t>(o->d_keys) & 15u) || (reinterpret_cast<uintptr_t>(o->d_values) & 15u))
    return TPZ_ERR_INVALID_ARG;
  TPZ_HIP(hipSetDevice(c->device));
  tpz_workspace* w = nullptr;
  {
    std::lock_guard<std::mutex> g(c->mu);
    tpz_err r = get_workspace(c, stream, b->n_blocks, &w);
    if (r != TPZ_SUCCESS) return r;
  }
  uint32_t* tail = w->d_tail;
  const uint64_t st = (uint64_t)b->n_blocks + 1;
  tpz::LaunchArgs a{};
  a.src = b->d_src;
  a.ext = b->d_ext;
  a.src_bytes = b->src_bytes;
  a.n_blocks = b->n_blocks;
  a.crc_tables = c->d_tables;
  a.data = nullptr;                 // no slots: every path writes the columns
  a.ends = o->d_ends;
  a.count = o->d_count;
  a.status = o->d_status;
  a.crc = o->d_crc;
  a.tail = tail;
  a.defer_count = tail + tpz::kTailBig;
  a.defer_list = w->d_defer + 4;
  a.spill_count = tail + tpz::kTailSpill;
  a.spill_list = w->d_defer + 4 + w->defer_cap;
  a.bw_count = tail + tpz::kTailBw;
  a.bw_list = nullptr;              // long blocks go to the spill path, which writes the columns
  a.rep = c->d_rep_tables;
  a.spill = o->d_spill;
  a.spill_cap = o->d_spill ? o->spill_cap : 0;
  a.spill_off = o->d_spill_off;
  a.spill_used = o->d_spill_used;
  a.num_cus = c->num_cus;
  a.big_scratch = w->d_big_scratch;
  a.big_grid = c->num_cus;
  a.efirst = o->d_first;
  a.keys = o->d_keys;
  a.vals = o->d_values;
  a.kfirst = o->d_first + st;
  a.vfirst = o->d_first + 2 * st;
  tpz::launch_decode(a, (hipStream_t)stream);
  TPZ_HIP(hipGetLastError());
  return TPZ_SUCCESS;
}

uint64_t tpz_layout_compress_bound(uint64_t src_bytes, uint64_t n_blocks) {
  return src_bytes + src_bytes / 6 + 40 * n_blocks + 64;
}

tpz_err tpz_compress_blocks(tpz_ctx* c, const tpz_batch* b, uint32_t codec, uint8_t* d_dst,
                            uint64_t* d_dst_ext, void* stream) {
  if (!c || !b || !d_dst_ext || (codec != 2 && codec != 3)) return TPZ_ERR_INVALID_ARG;
  if (b->n_blocks && (!b->d_src || !b->d_ext || !d_dst)) return TPZ_ERR_INVALID_ARG;
  // the match finder loads the blocks in aligned 16-byte pieces and the pack kernel stores them
  // the same way (tpz_compress.hip): both buffers 16-byte aligned, as tpz_decode_blocks_flat asks
  if (((uintptr_t)b->d_src | (uintptr_t)d_dst) & 15u) return TPZ_ERR_INVALID_ARG;
  TPZ_HIP(hipSetDevice(c->device));
  const uint64_t scratch = tpz::compress_scratch_bytes(b->src_bytes, b->n_blocks);
  const uint64_t parts = (uint64_t)tpz::flat_scan_parts_words(b->n_blocks);
  tpz_workspace* w = nullptr;
  {
    std::lock_guard<std::mutex> g(c->mu);
    w = &c->ws[stream];
    tpz_err r = grow(stream, &w->d_comp, &w->comp_cap, ((scratch + 15) & ~15ull) + 8 * parts);
    if (r != TPZ_SUCCESS) return r;
  }
  uint8_t* sc = static_cast<uint8_t*>(w->d_comp);
  tpz::launch_compress(b->d_src, b->d_ext, b->src_bytes, b->n_blocks, codec, sc, d_dst_ext,
                       reinterpret_cast<uint64_t*>(sc + ((scratch + 15) & ~15ull)), d_dst,
                       c->num_cus, (hipStream_t)stream);
  TPZ_HIP(hipGetLastError());
  return TPZ_SUCCESS;
}

tpz_err tpz_crc32_ranges(tpz_ctx* c, const tpz_batch* r, uint32_t* d_crc, void* stream) {
  return crc_ranges(c, r, 0, d_crc, nullptr, stream);
}

tpz_err tpz_verify_files(tpz_ctx* c, const tpz_batch* f, uint32_t* d_crc, uint8_t* d_status,
                         void* stream) {
  if (!d_status) return TPZ_ERR_INVALID_ARG;
  return crc_ranges(c, f, 4, d_crc, d_status, stream);
}

tpz_err tpz_verify_files_flat_layout(tpz_ctx* c, const tpz_batch* blocks,
                                     const uint32_t* d_file_block, const tpz_batch* tails,
                                     uint32_t* d_crc, uint8_t* d_status, uint64_t* d_first,
                                     void* stream) {
  if (!c || !blocks || !tails || !d_first || !d_file_block) return TPZ_ERR_INVALID_ARG;
  if (blocks->n_blocks && (!blocks->d_src || !blocks->d_ext ||
                           (reinterpret_cast<uintptr_t>(blocks->d_src) & 15u)))
    return TPZ_ERR_INVALID_ARG;
  if (tails->n_blocks && (!tails->d_src || !tails->d_ext || !d_crc || !d_status ||
                          (reinterpret_cast<uintptr_t>(tails->d_src) & 15u)))
    return TPZ_ERR_INVALID_ARG;
  if (blocks->n_blocks == 0 && tails->n_blocks == 0) {
    TPZ_HIP(hipSetDevice(c->device));
    TPZ_HIP(hipMemsetAsync(d_first, 0, 3 * 8, (hipStream_t)stream));
    return TPZ_SUCCESS;
  }
  TPZ_HIP(hipSetDevice(c->device));
  const uint64_t parts = tpz::flat_scan_parts_words(blocks->n_blocks);
  const uint64_t words = 2 * parts + blocks->n_blocks + tails->n_blocks;
  if (words > 0xFFFFFFFFull) return TPZ_ERR_INVALID_ARG;
  uint32_t* ws = nullptr;
  {
    std::lock_guard<std::mutex> g(c->mu);
    tpz_err e = get_acc(c, stream, (uint32_t)words, &ws);
    if (e != TPZ_SUCCESS) return e;
  }
  tpz::OpenLaunch a{};
  a.src = blocks->d_src;
  a.bext = blocks->d_ext;
  a.src_bytes = blocks->src_bytes;
  a.n_blocks = blocks->n_blocks;
  a.fblock = d_file_block;
  a.n_files = tails->n_blocks;
  a.tsrc = tails->d_src;
  a.text = tails->d_ext;
  a.first = d_first;
  a.part = reinterpret_cast<uint64_t*>(ws);
  a.cb = ws + 2 * parts;
  a.tacc = ws + 2 * parts + blocks->n_blocks;
  a.rep = c->d_rep_tables;
  a.tail_bytes = tails->src_bytes;
  if (tails->n_blocks)
    TPZ_HIP(hipMemsetAsync(a.tacc, 0, (size_t)tails->n_blocks * 4, (hipStream_t)stream));
  a.dtab = c->d_tables;
  a.rtab = c->d_range_tables;
  a.crc = d_crc;
  a.status = d_status;
  a.num_cus = c->num_cus;
  tpz::launch_open_flat(a, (hipStream_t)stream);
  TPZ_HIP(hipGetLastError());
  return TPZ_SUCCESS;
}

tpz_err tpz_seek_keys(tpz_ctx* c, const tpz_table* t, const uint8_t* d_keys,
                      const uint64_t* d_key_pos, uint32_t n_keys, uint32_t* d_block,
                      uint32_t* d_entry, uint8_t* d_status, uint8_t* d_valid, void* stream) {
  if (!c || !t || !d_key_pos || !d_block || !d_entry || !d_status || !d_valid)
    return TPZ_ERR_INVALID_ARG;
  if (n_keys == 0) return TPZ_SUCCESS;
  if (t->n_blocks && (!t->d_first_keys || !t->d_first_pos || !t->d_ext || !t->d_data ||
                      !t->d_ends || !t->d_count || !t->d_status))
    return TPZ_ERR_INVALID_ARG;
  TPZ_HIP(hipSetDevice(c->device));
  tpz::SeekLaunch a{t->d_first_keys, t->d_first_pos, t->n_blocks, t->d_ext, t->d_data,
                    t->d_ends, t->d_count, t->d_status, t->d_spill, t->d_spill_off, d_keys,
                    d_key_pos, n_keys, d_block, d_entry, d_status, d_valid,
                    t->d_entry_first};
  tpz::launch_seek(a, (hipStream_t)stream);
  TPZ_HIP(hipGetLastError());
  return TPZ_SUCCESS;
}

// Rust's saturating float-to-unsigned cast (`as u8`, `as usize`): NaN -> 0.
static uint64_t sat_cast(double x, double hi) {
  if (!(x == x) || x <= 0.0) return 0;
  return x >= hi ? (uint64_t)hi : (uint64_t)x;
}

tpz_err tpz_bloom_geometry(uint64_t n_keys, double fpp, uint64_t* filter_len, uint32_t* k) {
  if (!filter_len || !k || !(fpp >= 0.0 && fpp < 1.0)) return TPZ_ERR_INVALID_ARG;  // bloom.rs:49
  const double n = (double)n_keys;
  const double ln2sq = 0.6931471805599453 * 0.6931471805599453;   // LN_2.powi(2)
  const double m = -(n * std::log(fpp)) / ln2sq;
  if (std::isinf(m)) return TPZ_ERR_INVALID_ARG;   // fpp 0: the reference's `% limit` divides by 0
  uint64_t kk = sat_cast(std::ceil(m / n * ln2sq), 255.0);
  kk = kk < 1 ? 1 : (kk > 15 ? 15 : kk);
  *k = (uint32_t)kk;
  *filter_len = (sat_cast(std::ceil(m), 18446744073709549568.0) + 7) / 8 + 1;
  return TPZ_SUCCESS;
}

tpz_err tpz_bloom_build(tpz_ctx* c, const uint8_t* d_keys, const uint64_t* d_key_pos,
                        uint32_t n_keys, double fpp, uint8_t* d_filter, void* stream) {
  if (!c || !d_filter || (n_keys && !d_key_pos) || (reinterpret_cast<uintptr_t>(d_filter) & 3u))
    return TPZ_ERR_INVALID_ARG;
  uint64_t len = 0;
  uint32_t k = 0;
  tpz_err r = tpz_bloom_geometry(n_keys, fpp, &len, &k);
  if (r != TPZ_SUCCESS) return r;
  TPZ_HIP(hipSetDevice(c->device));
  hipStream_t s = (hipStream_t)stream;
  TPZ_HIP(hipMemsetAsync(d_filter, 0, (len + 3) & ~(uint64_t)3, s));
  static const bool atomic_only = std::getenv("TPZ_BLOOM_ATOMIC") != nullptr;   // A/B probe
  const uint64_t work = atomic_only ? 0 : tpz::bloom_build_work_bytes(n_keys, k, (len - 1) * 8);
  void* d_work = nullptr;
  if (work && n_keys) {   // the stream's grow-only scratch (stream-ordered reuse)
    std::lock_guard<std::mutex> g(c->mu);
    tpz_workspace& w = c->ws[stream];
    tpz_err r2 = grow(stream, &w.d_bloom, &w.bloom_cap, work);
    if (r2 != TPZ_SUCCESS) return r2;
    d_work = w.d_bloom;
  }
  tpz::BloomBuildLaunch a{d_keys, d_key_pos, n_keys, k, (len - 1) * 8, d_filter, (len + 3) / 4,
                          d_work};
  tpz::launch_bloom_build(a, s);
  TPZ_HIP(hipGetLastError());
  TPZ_HIP(hipMemsetAsync(d_filter + len - 1, (int)k, 1, s));        // the last byte is k
  return TPZ_SUCCESS;
}

tpz_err tpz_bloom_may_contain(tpz_ctx* c, const uint8_t* d_filter, uint64_t filter_len,
                              const uint8_t* d_keys, const uint64_t* d_key_pos, uint32_t n_keys,
                              uint8_t* d_out, void* stream) {
  if (!c || !d_key_pos || !d_out || (filter_len && !d_filter)) return TPZ_ERR_INVALID_ARG;
  if (n_keys == 0) return TPZ_SUCCESS;
  TPZ_HIP(hipSetDevice(c->device));
  tpz::BloomLaunch a{d_filter, filter_len, d_keys, d_key_pos, n_keys, d_out};
  tpz::launch_bloom(a, (hipStream_t)stream);
  TPZ_HIP(hipGetLastError());
  return TPZ_SUCCESS;
}


// The block plan on the stream, into info[0..3) = {most entries a block starting at any entry
// takes (>= the longest block), first entry the
// reference rejects (~0u: none), block count} (device memory, written by the kernels). With
// block_size <= kPlanBoundBlock no block holds more than kPlanChunk entries (each is >= 5 bytes), so
// the transfer tables are sized from that bound and the launch needs no host round trip; larger block
// sizes read the longest block back once (the chunk length follows it). *h_bad is set, and
// TPZ_ERR_INVALID_ARG returned, when that round trip finds a rejected entry.
static tpz_err plan_launch(tpz_ctx* c, const tpz_entries* en, uint32_t block_size, uint32_t* d_first,
                           uint64_t* d_ext, uint32_t* info, void* stream, uint64_t* h_bad) {
  hipStream_t s = (hipStream_t)stream;
  const uint32_t n = en->n_entries;
  std::unique_lock<std::mutex> lk(c->mu);
  tpz_workspace& w = c->ws[stream];
  lk.unlock();
  const size_t nwg = ((size_t)n + tpz::kPlanNextPer - 1) / tpz::kPlanNextPer;              // plan_next_kernel workgroups
  const size_t nx_words = (size_t)n + 2 * nwg + 2;           // nx, per-workgroup maxima and bad
  {
    std::lock_guard<std::mutex> g(c->mu);
    tpz_err r = grow(stream, &w.d_plan0, &w.plan0_cap, (nx_words + 4) * 4);
    if (r != TPZ_SUCCESS) return r;
  }
  uint32_t* nx = static_cast<uint32_t*>(w.d_plan0);
  tpz::PlanLaunch a{};
  a.phase = 0;
  a.kpos = en->d_kpos;
  a.vpos = en->d_vpos;
  a.n = n;
  a.block_size = block_size;
  a.nx = nx;
  a.info = info;
  a.first = d_first;
  a.ext = d_ext;
  TPZ_HIP(tpz::launch_plan(a, s));
  a.phase = 1;
  const uint32_t span = (block_size - 2) / 5 ? (block_size - 2) / 5 : 1u;   // entries per block <= span
  if (span <= tpz::kPlanChunk) {
    a.w = span;
    a.chunk = tpz::kPlanChunk;
  } else {
    uint32_t h_info[4];
    TPZ_HIP(hipMemcpyAsync(h_info, info, 16, hipMemcpyDeviceToHost, s));
    TPZ_HIP(hipStreamSynchronize(s));
    if (h_info[1] != 0xFFFFFFFFu) {
      *h_bad = h_info[1];
      return TPZ_ERR_INVALID_ARG;
    }
    a.w = h_info[0];
    a.chunk = a.w > tpz::kPlanChunk ? a.w : tpz::kPlanChunk;
  }
  const uint64_t K = (n + (uint64_t)a.chunk - 1) / a.chunk;
  {
    std::lock_guard<std::mutex> g(c->mu);
    tpz_err r = grow(stream, &w.d_plan1, &w.plan1_cap, (2 * K * a.w + K + 4) * 4);
    if (r != TPZ_SUCCESS) return r;
  }
  a.tab_a = static_cast<int*>(w.d_plan1);
  a.tab_b = a.tab_a + K * a.w;
  a.cnt = reinterpret_cast<uint32_t*>(a.tab_b + K * a.w);
  a.n_blocks = info + 2;
  TPZ_HIP(tpz::launch_plan(a, s));
  return TPZ_SUCCESS;
}

static bool plan_args_ok(const tpz_entries* en, uint32_t block_size) {
  return block_size > 2 && block_size <= 65536 && en->n_entries != 0xFFFFFFFFu &&
         (en->n_entries == 0 || (en->d_kpos && en->d_vpos));
}

tpz_err tpz_plan_blocks(tpz_ctx* c, const tpz_entries* en, uint32_t block_size, uint32_t* d_first,
                        uint64_t* d_ext, uint32_t* h_n_blocks, uint64_t* h_bad_entry,
                        void* stream) {
  if (!c || !en || !d_first || !d_ext || !h_n_blocks || !h_bad_entry) return TPZ_ERR_INVALID_ARG;
  *h_bad_entry = UINT64_MAX;
  *h_n_blocks = 0;
  if (!plan_args_ok(en, block_size)) return TPZ_ERR_INVALID_ARG;
  TPZ_HIP(hipSetDevice(c->device));
  hipStream_t s = (hipStream_t)stream;
  if (en->n_entries == 0) {  // SsTableBuilder with no entries: no block, an empty data region
    TPZ_HIP(hipMemsetAsync(d_first, 0, 4, s));
    TPZ_HIP(hipMemsetAsync(d_ext, 0, 8, s));
    TPZ_HIP(hipStreamSynchronize(s));
    return TPZ_SUCCESS;
  }
  // the stream's grow-only plan buffers; info sits after nx (one plan per stream at a time: the
  // call returns once the plan is done)
  tpz_err r = TPZ_SUCCESS;
  uint32_t* info = nullptr;
  uint32_t* h_info = nullptr;
  {
    std::lock_guard<std::mutex> g(c->mu);
    tpz_workspace& w = c->ws[stream];
    const size_t nwg = ((size_t)en->n_entries + tpz::kPlanNextPer - 1) / tpz::kPlanNextPer;
    r = grow(stream, &w.d_plan0, &w.plan0_cap, ((size_t)en->n_entries + 2 * nwg + 2 + 4) * 4);
    if (r == TPZ_SUCCESS)
      info = static_cast<uint32_t*>(w.d_plan0) + (size_t)en->n_entries + 2 * nwg + 2;
    if (r == TPZ_SUCCESS && !w.h_info && hipHostMalloc(&w.h_info, 16) != hipSuccess) {
      w.h_info = nullptr;
      r = TPZ_ERR_NOMEM;
    }
    h_info = w.h_info;
  }
  if (r != TPZ_SUCCESS) return r;
  r = plan_launch(c, en, block_size, d_first, d_ext, info, stream, h_bad_entry);
  if (r != TPZ_SUCCESS) return r;
  TPZ_HIP(hipMemcpyAsync(h_info, info, 16, hipMemcpyDeviceToHost, s));   // one round trip
  TPZ_HIP(hipStreamSynchronize(s));
  if (h_info[1] != 0xFFFFFFFFu) {
    *h_bad_entry = h_info[1];
    return TPZ_ERR_INVALID_ARG;
  }
  *h_n_blocks = h_info[2];
  return TPZ_SUCCESS;
}

tpz_err tpz_plan_blocks_async(tpz_ctx* c, const tpz_entries* en, uint32_t block_size,
                              uint32_t* d_first, uint64_t* d_ext, uint32_t* d_info, void* stream) {
  if (!c || !en || !d_first || !d_ext || !d_info) return TPZ_ERR_INVALID_ARG;
  if (!plan_args_ok(en, block_size)) return TPZ_ERR_INVALID_ARG;
  TPZ_HIP(hipSetDevice(c->device));
  hipStream_t s = (hipStream_t)stream;
  if (en->n_entries == 0) {
    TPZ_HIP(hipMemsetAsync(d_first, 0, 4, s));
    TPZ_HIP(hipMemsetAsync(d_ext, 0, 8, s));
    TPZ_HIP(hipMemsetAsync(d_info, 0, 16, s));
    TPZ_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d_info + 1), 0xFFFFFFFFu, 1, s));
    return TPZ_SUCCESS;
  }
  uint64_t h_bad = UINT64_MAX;
  const tpz_err r = plan_launch(c, en, block_size, d_first, d_ext, d_info, stream, &h_bad);
  // a rejected entry found by the round trip of a large block size: the kernels have written
  // d_info[1] already, and the plan stops there (d_info[2] stays 0)
  if (r == TPZ_ERR_INVALID_ARG && h_bad != UINT64_MAX) {
    TPZ_HIP(hipMemsetAsync(d_info + 2, 0, 4, s));
    return TPZ_SUCCESS;
  }
  return r;
}

static tpz_err encode_launch(tpz_ctx* c, const tpz_entries* en, const uint32_t* d_first,
                             const uint64_t* d_ext, uint32_t n_blocks, const uint32_t* d_info,
                             uint8_t* d_out, void* stream) {
  if ((reinterpret_cast<uintptr_t>(d_out) & 15u) || !en->d_kpos || !en->d_vpos ||
      (!en->d_keys && en->key_bytes) || (!en->d_vals && en->val_bytes))
    return TPZ_ERR_INVALID_ARG;
  TPZ_HIP(hipSetDevice(c->device));
  hipStream_t s = (hipStream_t)stream;
  tpz_workspace* w = nullptr;    // the big-block worklist: the stream's decode worklist
  {
    std::lock_guard<std::mutex> g(c->mu);
    tpz_err r = get_workspace(c, stream, n_blocks, &w);
    if (r != TPZ_SUCCESS) return r;
  }
  tpz::EncodeLaunch a{};
  a.keys = en->d_keys;
  a.kpos = en->d_kpos;
  a.key_bytes = en->key_bytes;
  a.vals = en->d_vals;
  a.vpos = en->d_vpos;
  a.val_bytes = en->val_bytes;
  a.first = d_first;
  a.ext = d_ext;
  a.n_blocks = n_blocks;
  a.plan_info = d_info;
  a.crc_tables = c->d_tables;
  a.out = d_out;
  a.big_count = w->d_defer;
  a.big_list = w->d_defer + 4;
  a.num_cus = c->num_cus;
  TPZ_HIP(tpz::launch_encode(a, s));
  return TPZ_SUCCESS;
}

tpz_err tpz_encode_blocks(tpz_ctx* c, const tpz_entries* en, const uint32_t* d_first,
                          const uint64_t* d_ext, uint32_t n_blocks, uint8_t* d_out, void* stream) {
  if (!c || !en || !d_first || !d_ext || !d_out) return TPZ_ERR_INVALID_ARG;
  if (n_blocks == 0) return TPZ_SUCCESS;
  return encode_launch(c, en, d_first, d_ext, n_blocks, nullptr, d_out, stream);
}

tpz_err tpz_encode_blocks_async(tpz_ctx* c, const tpz_entries* en, const uint32_t* d_first,
                                const uint64_t* d_ext, const uint32_t* d_info, uint8_t* d_out,
                                void* stream) {
  if (!c || !en || !d_first || !d_ext || !d_info || !d_out) return TPZ_ERR_INVALID_ARG;
  if (en->n_entries == 0) return TPZ_SUCCESS;
  // at most one block per entry: the worklist bound
  return encode_launch(c, en, d_first, d_ext, en->n_entries, d_info, d_out, stream);
}

tpz_err tpz_pack_ends(tpz_ctx* c, const tpz_batch* b, const tpz_columns* cols,
                      const uint64_t* d_first, uint32_t* d_dense, void* stream) {
  if (!c || !b || !cols || !d_first || !d_dense) return TPZ_ERR_INVALID_ARG;
  if (b->n_blocks == 0) return TPZ_SUCCESS;
  if (!b->d_ext || !cols->d_ends || !cols->d_count || !cols->d_status) return TPZ_ERR_INVALID_ARG;
  TPZ_HIP(hipSetDevice(c->device));
  tpz::PackLaunch a{b->d_ext, b->n_blocks, cols->d_ends, cols->d_count, cols->d_status,
                    cols->d_spill, cols->d_spill_off, d_first, d_dense, cols->d_entry_first};
  tpz::launch_pack_ends(a, (hipStream_t)stream);
  TPZ_HIP(hipGetLastError());
  return TPZ_SUCCESS;
}

uint64_t tpz_host_xxh3_64(const uint8_t* h_buf, uint64_t len) {
  return tpz::xxh3::hash64(h_buf, len);
}

int tpz_format_block_error(int status, uint32_t crc_expected, uint32_t crc_actual, char* buf,
                           size_t cap) {
  char tmp[96];
  switch (status) {
    case TPZ_BLOCK_OK: tmp[0] = 0; break;
    case TPZ_BLOCK_EMPTY: std::snprintf(tmp, sizeof tmp, "data is empty"); break;   // compress.rs:97
    case TPZ_BLOCK_BAD_TAG: std::snprintf(tmp, sizeof tmp, "invaild data"); break;  // compress.rs:102
    case TPZ_BLOCK_UNSUPPORTED_CODEC: std::snprintf(tmp, sizeof tmp, "unsupported codec"); break;
    case TPZ_BLOCK_CHECKSUM_MISMATCH:                                                // checksum.rs:17-20
      std::snprintf(tmp, sizeof tmp, "checksum: expected %u, actual %u", crc_expected, crc_actual);
      break;
    case TPZ_BLOCK_MALFORMED: std::snprintf(tmp, sizeof tmp, "malformed block"); break;
    case TPZ_BLOCK_OK_SPILLED: tmp[0] = 0; break;   // Ok(Block), decoded into the spill arena
    case TPZ_BLOCK_SPILL_FULL: std::snprintf(tmp, sizeof tmp, "spill arena too small"); break;
    case TPZ_BLOCK_CODEC_ERROR: std::snprintf(tmp, sizeof tmp, "decompression failed"); break;
    case TPZ_BLOCK_BAD_ENTRY: tmp[0] = 0; break;    // Ok(Block); its bad entries panic on access
    default: std::snprintf(tmp, sizeof tmp, "unknown status %d", status); break;
  }
  int n = (int)std::strlen(tmp);
  if (buf && cap) {
    std::strncpy(buf, tmp, cap - 1);
    buf[cap - 1] = 0;
  }
  return n;
}

}  // extern "C"
