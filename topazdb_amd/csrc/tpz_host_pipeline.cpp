// tpz_host_pipeline.cpp — tpz_decode_blocks_host: the read path from host memory.
//
// topazdb reads a block with one pread into a fresh Vec (FileObject::read,
// src/table/file_object.rs:23-27) and decodes it on the CPU (SsTable::read_block,
// src/table.rs:154-164). Here a whole run of blocks in host memory goes through the device:
// chunks of blocks are uploaded, decoded (tpz_decode_blocks), their entry ends packed
// (tpz_pack_ends) and every output copied back, on two streams so that chunk k+1's upload and
// decode overlap chunk k's downloads.
//
// Chunk geometry. A chunk of blocks [lo, hi) is uploaded to a device buffer whose byte 0 stands
// for host byte B = ext[lo] rounded down to a multiple of 384 (= lcm(128, 96)); its extents are
// ext[i] - B. Because B is a multiple of 128 and of 96, the chunk's slot bases and entry bases
// are the whole batch's shifted by constants (tpz_slot_base(e - B, i - lo) =
// tpz_slot_base(e, i) - B - 256 lo), so the chunk's slots land in h_data exactly where
// tpz_decode_blocks would put them for the whole batch. Only the chunk's own bytes
// [ext[lo], ext[hi]) are uploaded; the decode never reads the bytes of the device buffer before
// the chunk's first block (the first 16-byte piece is masked, tpz_decode.hip zero_head).
//
// Three streams and three buffer slots, so that the two copy directions run at once:
//   up:    H2D of chunk k's blocks and extents (after chunk k-3's downloads freed its slot)
//   comp:  decode, the entry prefix (count_prefix_kernel), D2H of the per-block metadata;
//          later, once the host has placed the chunk, tpz_pack_ends
//   down:  D2H of the slots, the packed ends and the spill records
// The host waits only for chunk k's metadata (entry total, spill bytes), while chunk k+1 uploads
// and chunk k-1 downloads; a spill arena that overflowed is grown and the chunk decoded again.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "tpz_internal.h"

namespace {

struct Buf {
  void* p = nullptr;
  size_t n = 0;
  bool host = false;
  ~Buf() { release(); }
  void release() {
    if (p) (void)(host ? hipHostFree(p) : hipFree(p));
    p = nullptr;
    n = 0;
  }
  hipError_t ensure(size_t bytes) {
    if (bytes <= n) return hipSuccess;
    release();
    const size_t b = std::max<size_t>(bytes, 256);
    hipError_t e = host ? hipHostMalloc(&p, b, hipHostMallocDefault) : hipMalloc(&p, b);
    if (e == hipSuccess) n = b;
    return e;
  }
  template <class T> T* as() const { return static_cast<T*>(p); }
};

// A caller range page-locked for the call (if it was not already).
struct Pin {
  void* p = nullptr;
  ~Pin() {
    if (p) (void)hipHostUnregister(p);
  }
  void pin(const void* q, size_t bytes) {
    if (!q || !bytes) return;
    if (hipHostRegister(const_cast<void*>(q), bytes, hipHostRegisterDefault) == hipSuccess)
      p = const_cast<void*>(q);
    else
      (void)hipGetLastError();   // already pinned (or not pinnable): plain copies still work
  }
};

struct Slot {
  hipEvent_t ev = nullptr;        // metadata landed (comp)
  hipEvent_t ev_up = nullptr;     // blocks uploaded (up)
  hipEvent_t ev_pack = nullptr;   // ends packed (comp)
  hipEvent_t ev_down = nullptr;   // downloads done: the slot is free (down)
  bool used = false;
  Buf d_src, d_ext, d_data, d_ends, d_count, d_status, d_crc, d_spill, d_spill_off, d_used,
      d_first, d_dense;
  Buf h_ext, h_first, h_count, h_status, h_crc, h_spill_off, h_used;
  uint32_t lo = 0, hi = 0;
  uint64_t base = 0;   // host byte of device byte 0 (a multiple of 384)
  Slot() {
    h_ext.host = h_first.host = h_count.host = h_status.host = h_crc.host = h_spill_off.host =
        h_used.host = true;
  }
  ~Slot() {
    for (hipEvent_t e : {ev, ev_up, ev_pack, ev_down})
      if (e) (void)hipEventDestroy(e);
  }
};

#define PIPE_HIP(call)                                                         \
  do {                                                                         \
    hipError_t e_ = (call);                                                    \
    if (e_ != hipSuccess) return tpz_internal_hip_fail(e_, #call);             \
  } while (0)

}  // namespace

extern "C" tpz_err tpz_decode_blocks_host(tpz_ctx* ctx, const uint8_t* h_src,
                                          const uint64_t* h_ext, uint32_t n,
                                          const tpz_host_columns* o, uint32_t chunk_blocks) {
  if (!ctx || !h_ext || !o || !o->h_first || !o->h_count || !o->h_status || !o->h_crc ||
      !o->h_spill_off || !o->h_spill_used || (n && (!h_src || !o->h_data)) ||
      (o->ends_cap && !o->h_ends) || (o->spill_cap && !o->h_spill))
    return TPZ_ERR_INVALID_ARG;
  for (uint32_t i = 0; i < n; i++)
    if (h_ext[i + 1] < h_ext[i]) return TPZ_ERR_INVALID_ARG;
  o->h_first[0] = 0;
  *o->h_spill_used = 0;
  if (n == 0) return TPZ_SUCCESS;
  PIPE_HIP(hipSetDevice(tpz_internal_device(ctx)));
  const uint32_t cb = chunk_blocks ? chunk_blocks : 8192u;
  const uint64_t src_bytes = h_ext[n];

  // the largest chunk's byte span (from its 384-aligned base)
  uint64_t max_span = 0;
  for (uint32_t lo = 0; lo < n; lo += cb) {
    const uint32_t hi = std::min(n, lo + cb);
    max_span = std::max<uint64_t>(max_span, h_ext[hi] - (h_ext[lo] - h_ext[lo] % 384));
  }
  Pin pin_src, pin_data, pin_ends, pin_spill;
  pin_src.pin(h_src + h_ext[0], h_ext[n] - h_ext[0]);
  pin_data.pin(o->h_data, tpz_data_capacity(src_bytes, n));
  pin_ends.pin(o->h_ends, o->ends_cap * 4);
  pin_spill.pin(o->h_spill, o->spill_cap);

  struct Streams {
    hipStream_t up = nullptr, comp = nullptr, down = nullptr;
    ~Streams() {
      for (hipStream_t q : {up, comp, down})
        if (q) (void)hipStreamDestroy(q);
    }
  } st;
  PIPE_HIP(hipStreamCreateWithFlags(&st.up, hipStreamNonBlocking));
  PIPE_HIP(hipStreamCreateWithFlags(&st.comp, hipStreamNonBlocking));
  PIPE_HIP(hipStreamCreateWithFlags(&st.down, hipStreamNonBlocking));
  constexpr int kSlots = 3;
  Slot slot[kSlots];
  for (Slot& S : slot) {
    for (hipEvent_t* e : {&S.ev, &S.ev_up, &S.ev_pack, &S.ev_down})
      PIPE_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
    const uint64_t m = std::min<uint64_t>(cb, n);
    PIPE_HIP(S.d_src.ensure(max_span + 16));
    PIPE_HIP(S.d_ext.ensure((m + 1) * 8));
    PIPE_HIP(S.d_data.ensure(tpz_data_capacity(max_span, m)));
    PIPE_HIP(S.d_ends.ensure(2 * tpz_entry_capacity(max_span, m) * 4));
    PIPE_HIP(S.d_count.ensure(m * 4));
    PIPE_HIP(S.d_status.ensure(m));
    PIPE_HIP(S.d_crc.ensure(m * 4));
    PIPE_HIP(S.d_spill_off.ensure(m * 8));
    PIPE_HIP(S.d_used.ensure(8));
    PIPE_HIP(S.d_first.ensure((m + 1) * 8));
    PIPE_HIP(S.d_dense.ensure(2 * tpz_entry_capacity(max_span, m) * 4));
    PIPE_HIP(S.h_ext.ensure((m + 1) * 8));
    PIPE_HIP(S.h_first.ensure((m + 1) * 8));
    PIPE_HIP(S.h_count.ensure(m * 4));
    PIPE_HIP(S.h_status.ensure(m));
    PIPE_HIP(S.h_crc.ensure(m * 4));
    PIPE_HIP(S.h_spill_off.ensure(m * 8));
    PIPE_HIP(S.h_used.ensure(8));
  }

  // upload + decode + entry prefix + metadata download of the chunk in S (lo/hi/base set)
  auto decode_chunk = [&](Slot& S) -> tpz_err {
    const uint32_t m = S.hi - S.lo;
    const uint64_t span = h_ext[S.hi] - S.base;
    tpz_columns cols{};
    cols.d_data = S.d_data.as<uint8_t>();
    cols.d_ends = S.d_ends.as<uint32_t>();
    cols.d_count = S.d_count.as<uint32_t>();
    cols.d_status = S.d_status.as<uint8_t>();
    cols.d_crc = S.d_crc.as<uint32_t>();
    cols.d_spill = S.d_spill.n ? S.d_spill.as<uint8_t>() : nullptr;
    cols.spill_cap = S.d_spill.n;
    cols.d_spill_off = S.d_spill_off.as<uint64_t>();
    cols.d_spill_used = S.d_used.as<uint64_t>();
    const tpz_batch b{S.d_src.as<uint8_t>(), S.d_ext.as<uint64_t>(), m, span};
    PIPE_HIP(hipStreamWaitEvent(st.comp, S.ev_up, 0));
    tpz_err r = tpz_decode_blocks(ctx, &b, &cols, st.comp);
    if (r != TPZ_SUCCESS) return r;
    tpz::launch_count_prefix(cols.d_count, cols.d_status, m, S.d_first.as<uint64_t>(), st.comp);
    PIPE_HIP(hipGetLastError());
    PIPE_HIP(hipMemcpyAsync(S.h_first.p, S.d_first.p, (m + 1) * 8, hipMemcpyDeviceToHost, st.comp));
    PIPE_HIP(hipMemcpyAsync(S.h_count.p, S.d_count.p, m * 4, hipMemcpyDeviceToHost, st.comp));
    PIPE_HIP(hipMemcpyAsync(S.h_status.p, S.d_status.p, m, hipMemcpyDeviceToHost, st.comp));
    PIPE_HIP(hipMemcpyAsync(S.h_crc.p, S.d_crc.p, m * 4, hipMemcpyDeviceToHost, st.comp));
    PIPE_HIP(hipMemcpyAsync(S.h_spill_off.p, S.d_spill_off.p, m * 8, hipMemcpyDeviceToHost, st.comp));
    PIPE_HIP(hipMemcpyAsync(S.h_used.p, S.d_used.p, 8, hipMemcpyDeviceToHost, st.comp));
    PIPE_HIP(hipEventRecord(S.ev, st.comp));
    return TPZ_SUCCESS;
  };

  auto issue = [&](Slot& S, uint32_t lo) -> tpz_err {
    if (S.used) {
      // the slot's previous chunk: its downloads must be done before the upload overwrites the
      // device buffers (a stream wait), and its extents upload before h_ext is rewritten (long
      // done; its metadata was consumed by finish())
      PIPE_HIP(hipStreamWaitEvent(st.up, S.ev_down, 0));
      PIPE_HIP(hipEventSynchronize(S.ev_up));
    }
    S.used = true;
    S.lo = lo;
    S.hi = std::min(n, lo + cb);
    S.base = h_ext[lo] - h_ext[lo] % 384;
    uint64_t* e = S.h_ext.as<uint64_t>();
    for (uint32_t i = S.lo; i <= S.hi; i++) e[i - S.lo] = h_ext[i] - S.base;
    const uint64_t off = h_ext[lo] - S.base;
    PIPE_HIP(hipMemcpyAsync(S.d_src.as<uint8_t>() + off, h_src + h_ext[lo], h_ext[S.hi] - h_ext[lo],
                            hipMemcpyHostToDevice, st.up));
    PIPE_HIP(hipMemcpyAsync(S.d_ext.p, S.h_ext.p, (S.hi - S.lo + 1) * 8, hipMemcpyHostToDevice,
                            st.up));
    PIPE_HIP(hipEventRecord(S.ev_up, st.up));
    return decode_chunk(S);
  };

  uint64_t g_first = 0, g_spill = 0;
  bool short_ends = false, short_spill = false;
  auto finish = [&](Slot& S) -> tpz_err {
    PIPE_HIP(hipEventSynchronize(S.ev));
    const uint32_t m = S.hi - S.lo;
    uint64_t used = *S.h_used.as<uint64_t>();
    if (used > S.d_spill.n) {                 // the spill arena overflowed: grow, decode again
      PIPE_HIP(hipStreamSynchronize(st.comp));
      PIPE_HIP(S.d_spill.ensure(used + (used >> 2)));
      tpz_err r = decode_chunk(S);
      if (r != TPZ_SUCCESS) return r;
      PIPE_HIP(hipEventSynchronize(S.ev));
      used = *S.h_used.as<uint64_t>();
    }
    const uint64_t* first = S.h_first.as<uint64_t>();
    const uint64_t total = first[m];
    const uint64_t span = h_ext[S.hi] - S.base;
    // the chunk's own slots, into the batch's slotted layout
    const uint64_t d0 = tpz_slot_base(h_ext[S.lo] - S.base, 0);
    const uint64_t d1 = tpz_slot_base(span, m);
    const uint64_t h0 = tpz_slot_base(h_ext[S.lo], S.lo);
    PIPE_HIP(hipStreamWaitEvent(st.down, S.ev, 0));
    PIPE_HIP(hipMemcpyAsync(o->h_data + h0, S.d_data.as<uint8_t>() + d0, d1 - d0,
                            hipMemcpyDeviceToHost, st.down));
    // the used entry ends, packed
    if (2 * (g_first + total) <= o->ends_cap) {
      if (2 * total * 4 > S.d_dense.n) {      // only spilled blocks can exceed the slot bound
        PIPE_HIP(hipStreamSynchronize(st.comp));
        PIPE_HIP(hipStreamSynchronize(st.down));
        PIPE_HIP(S.d_dense.ensure(2 * total * 4));
      }
      tpz_columns cols{};
      cols.d_ends = S.d_ends.as<uint32_t>();
      cols.d_count = S.d_count.as<uint32_t>();
      cols.d_status = S.d_status.as<uint8_t>();
      cols.d_spill = S.d_spill.n ? S.d_spill.as<uint8_t>() : nullptr;
      cols.d_spill_off = S.d_spill_off.as<uint64_t>();
      const tpz_batch b{S.d_src.as<uint8_t>(), S.d_ext.as<uint64_t>(), m, span};
      tpz_err r = tpz_pack_ends(ctx, &b, &cols, S.d_first.as<uint64_t>(), S.d_dense.as<uint32_t>(),
                                st.comp);
      if (r != TPZ_SUCCESS) return r;
      PIPE_HIP(hipEventRecord(S.ev_pack, st.comp));
      PIPE_HIP(hipStreamWaitEvent(st.down, S.ev_pack, 0));
      if (total)
        PIPE_HIP(hipMemcpyAsync(o->h_ends + 2 * g_first, S.d_dense.p, 2 * total * 4,
                                hipMemcpyDeviceToHost, st.down));
    } else {
      short_ends = true;
    }
    // the spill records
    if (g_spill + used <= o->spill_cap) {
      if (used)
        PIPE_HIP(hipMemcpyAsync(o->h_spill + g_spill, S.d_spill.p, used, hipMemcpyDeviceToHost,
                                st.down));
    } else {
      short_spill = true;
    }
    // per-block metadata
    const uint8_t* bst = S.h_status.as<uint8_t>();
    const uint64_t* soff = S.h_spill_off.as<uint64_t>();
    std::memcpy(o->h_count + S.lo, S.h_count.p, m * 4);
    std::memcpy(o->h_status + S.lo, S.h_status.p, m);
    std::memcpy(o->h_crc + S.lo, S.h_crc.p, m * 4);
    for (uint32_t j = 0; j < m; j++) {
      o->h_first[S.lo + j] = g_first + first[j];
      if (tpz::block_in_spill(bst[j])) o->h_spill_off[S.lo + j] = g_spill + soff[j];
    }
    g_first += total;
    g_spill += used;
    o->h_first[S.hi] = g_first;
    *o->h_spill_used = g_spill;
    PIPE_HIP(hipEventRecord(S.ev_down, st.down));
    return TPZ_SUCCESS;
  };

  // chunk k is issued, then chunk k-1 finished: the host waits for k-1's metadata while k
  // uploads and k-2 downloads
  const uint32_t n_chunks = (n + cb - 1) / cb;
  for (uint32_t k = 0; k <= n_chunks; k++) {
    if (k < n_chunks) {
      tpz_err r = issue(slot[k % kSlots], k * cb);
      if (r != TPZ_SUCCESS) return r;
    }
    if (k >= 1) {
      tpz_err r = finish(slot[(k - 1) % kSlots]);
      if (r != TPZ_SUCCESS) return r;
    }
  }
  PIPE_HIP(hipStreamSynchronize(st.up));
  PIPE_HIP(hipStreamSynchronize(st.comp));
  PIPE_HIP(hipStreamSynchronize(st.down));
  return (short_ends || short_spill) ? TPZ_ERR_NOMEM : TPZ_SUCCESS;
}
