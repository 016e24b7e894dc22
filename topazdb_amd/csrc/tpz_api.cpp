// tpz_api.cpp — the C ABI of include/tpz_gpu.h: context, workspace, launches, error text.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "tpz_internal.h"

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

}  // namespace

// Device workspace of one stream: the big-path worklist (counter + list) and the big path's
// per-workgroup entry tables. Decodes on different streams run concurrently, so each stream
// has its own; decodes on one stream are ordered by the stream.
struct tpz_workspace {
  uint32_t* d_defer = nullptr;  // [0] = counter, [1..] = list
  uint32_t defer_cap = 0;
  uint64_t* d_big_scratch = nullptr;
};

struct tpz_ctx {
  int device = 0;
  uint32_t num_cus = 0;
  uint32_t* d_tables = nullptr;
  std::mutex mu;  // guards the workspace map
  std::unordered_map<void*, tpz_workspace> ws;
};

namespace {

void free_workspace(tpz_workspace& w) {
  if (w.d_defer) (void)hipFree(w.d_defer);
  if (w.d_big_scratch) (void)hipFree(w.d_big_scratch);
  w = tpz_workspace{};
}

// The stream's workspace, grown to max_blocks. Caller holds c->mu.
tpz_err get_workspace(tpz_ctx* c, void* stream, uint32_t max_blocks, tpz_workspace** out) {
  tpz_workspace& w = c->ws[stream];
  if (!w.d_big_scratch)
    TPZ_HIP(hipMalloc(&w.d_big_scratch, (size_t)c->num_cus * 2 * tpz::kBigMaxSlots * sizeof(uint64_t)));
  if (!w.d_defer || w.defer_cap < max_blocks) {
    uint32_t* d = nullptr;
    TPZ_HIP(hipMalloc(&d, ((size_t)max_blocks + 1) * 4));
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

extern "C" {

uint64_t tpz_layout_key_base(uint64_t ext_i, uint64_t i) { return tpz_key_base(ext_i, i); }
uint64_t tpz_layout_entry_base(uint64_t ext_i, uint64_t i) { return tpz_entry_base(ext_i, i); }
uint64_t tpz_layout_col_capacity(uint64_t s, uint64_t n) { return tpz_col_capacity(s, n); }
uint64_t tpz_layout_entry_capacity(uint64_t s, uint64_t n) { return tpz_entry_capacity(s, n); }

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
  std::vector<uint32_t> t = build_crc_tables();
  hipError_t e = hipMalloc(&c->d_tables, t.size() * 4);
  if (e == hipSuccess) e = hipMemcpy(c->d_tables, t.data(), t.size() * 4, hipMemcpyHostToDevice);
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
  for (auto& kv : c->ws) free_workspace(kv.second);
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
  if (b->n_blocks == 0) return TPZ_SUCCESS;
  if (!b->d_src || !b->d_ext || !o->d_keys || !o->d_vals || !o->d_ends || !o->d_count ||
      !o->d_status || !o->d_crc)
    return TPZ_ERR_INVALID_ARG;
  TPZ_HIP(hipSetDevice(c->device));
  tpz_workspace* w = nullptr;
  {
    std::lock_guard<std::mutex> g(c->mu);
    tpz_err r = get_workspace(c, stream, b->n_blocks, &w);
    if (r != TPZ_SUCCESS) return r;
  }
  hipStream_t s = (hipStream_t)stream;
  TPZ_HIP(hipMemsetAsync(w->d_defer, 0, 4, s));
  tpz::LaunchArgs a{};
  a.src = b->d_src;
  a.ext = b->d_ext;
  a.src_bytes = b->src_bytes;
  a.n_blocks = b->n_blocks;
  a.crc_tables = c->d_tables;
  a.keys = o->d_keys;
  a.vals = o->d_vals;
  a.ends = o->d_ends;
  a.count = o->d_count;
  a.status = o->d_status;
  a.crc = o->d_crc;
  a.defer_count = w->d_defer;
  a.defer_list = w->d_defer + 1;
  a.num_cus = c->num_cus;
  a.big_scratch = w->d_big_scratch;
  a.big_grid = c->num_cus;
  tpz::launch_decode(a, s);
  TPZ_HIP(hipGetLastError());
  return TPZ_SUCCESS;
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
    case TPZ_BLOCK_OVERLAP: std::snprintf(tmp, sizeof tmp, "overlapping entries"); break;
    case TPZ_BLOCK_TOO_LARGE: std::snprintf(tmp, sizeof tmp, "block too large"); break;
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
