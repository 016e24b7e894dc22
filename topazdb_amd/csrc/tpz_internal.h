// tpz_internal.h — shared between the C ABI (tpz_api.cpp) and the kernels (tpz_decode.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tpz_gpu.h"

// Context accessors for the host pipeline (tpz_host_pipeline.cpp; defined in tpz_api.cpp).
int tpz_internal_device(tpz_ctx* c);
tpz_err tpz_internal_hip_fail(hipError_t e, const char* what);
// Sets tpz_last_error's text and returns err.
tpz_err tpz_internal_fail(tpz_err err, const char* what);
// The context's pool of host pipelines (streams + buffers of tpz_decode_blocks_host, reused
// across calls; one per concurrent caller): acquire returns a free one or nullptr; release puts
// one back (fresh = created by this call: the context takes ownership); the context destroys
// them with tpz_internal_pipe_destroy (tpz_host_pipeline.cpp).
void* tpz_internal_pipe_acquire(tpz_ctx* c);
void tpz_internal_pipe_release(tpz_ctx* c, void* pipe, bool fresh);
void tpz_internal_pipe_destroy(void* pipe);

namespace tpz {

// CRC-32 lookup tables of the block decode, uploaded once per context (tpz_api.cpp):
// ids 0..15 = T_0..T_15 (slice-by-16); ids 16+4j+i = T_{n_j-1-i}: the shift-by-n_j operator,
// n_j = kCrcShiftBytes[j] = 80 * 2^j (the lane-position shifts of the CRC combine; 2 x 2560 B
// chains the 5120-B super-rounds of long blocks);
// id 40 = kCrcInvTable: inv[t] = the byte b whose T_0[b] has top byte t (one zero byte un-shifted).
constexpr int kNumCrcTables = 41;
constexpr int kCrcInvTable = 40;
constexpr int kCrcLaneBytes = 80;
constexpr int kCrcShiftBytes[6] = {80, 160, 320, 640, 1280, 2560};
// Big path entry-table capacity per block and column: slots are only written when 6n <= len
// (the unified key+value table holds 2 x this).
constexpr uint32_t kBigMaxSlots = TPZ_LDS_BLOCK_BYTES / 6 + 16;

// Range CRC (tpz_crc.hip): shift-by-16*2^j operators j = 0..kRangeShiftOps-1 in the global
// range tables (ranges up to 16 * 2^kRangeShiftOps bytes), and the 32-fold replicated
// slice-by-4 table (4 x 256 x 32 u32).
constexpr int kRangeShiftOps = 32;
constexpr int kRangeTables = 16 + 4 * kRangeShiftOps;
// ... followed by 4 power tables: id kPowTable + i, entry j = x^(8 j 256^i) mod P (the shift by
// j * 256^i bytes as a GF(2)[x] factor: tpz_flat.hip open_finish_kernel)
constexpr int kPowTable = kRangeTables;
constexpr int kRangeTablesAll = kRangeTables + 4;
constexpr int kCrcRepWords = 4 * 256 * 32;

// Slotted layout (include/tpz_gpu.h), callable from device code.
__host__ __device__ inline uint64_t slot_base(uint64_t ext_i, uint64_t i) {
  return ((ext_i + 127u) & ~(uint64_t)127u) + 256u * i;
}
__host__ __device__ inline uint64_t entry_base(uint64_t ext_i, uint64_t i) {
  return 16u * (ext_i / 96u + i);
}
__host__ __device__ inline uint64_t value_start(uint64_t key_bytes) {
  return (key_bytes + 15u) & ~(uint64_t)15u;
}
// Spill records (include/tpz_gpu.h): u32 ends[2n], then the stream from spill_stream(n).
__host__ __device__ inline uint64_t spill_stream(uint64_t n) {
  return (8u * n + 127u) & ~(uint64_t)127u;
}
__host__ __device__ inline uint64_t spill_record_bytes(uint64_t n, uint64_t k, uint64_t v) {
  return spill_stream(n) + ((value_start(k) + v + 127u) & ~(uint64_t)127u);
}
// A TPZ_BLOCK_BAD_ENTRY record's class bytes follow its ends and stream.
__host__ __device__ inline uint64_t spill_classes(uint64_t n, uint64_t k, uint64_t v) {
  return spill_record_bytes(n, k, v);
}
// Readers of decoded blocks: a block whose entries are in its slot or in a spill record.
__host__ __device__ inline bool block_decoded(uint32_t st) {
  return st == TPZ_BLOCK_OK || st == TPZ_BLOCK_OK_SPILLED || st == TPZ_BLOCK_BAD_ENTRY;
}
__host__ __device__ inline bool block_in_spill(uint32_t st) {
  return st == TPZ_BLOCK_OK_SPILLED || st == TPZ_BLOCK_BAD_ENTRY;
}

struct LaunchArgs {
  const uint8_t* src;
  const uint64_t* ext;
  uint64_t src_bytes;
  uint32_t n_blocks;
  const uint32_t* crc_tables;
  uint8_t* data;
  uint32_t* ends;
  uint32_t* count;
  uint8_t* status;
  uint32_t* crc;
  uint32_t* defer_list;   // workspace: n_blocks entries
  uint32_t* defer_count;  // tail + kTailBig
  uint32_t num_cus;
  uint64_t* big_scratch;  // big_grid x 2 x kBigMaxSlots
  uint32_t big_grid;
  uint32_t* spill_list;   // workspace: n_blocks entries (blocks for the spill path)
  uint32_t* spill_count;  // tail + kTailSpill
  uint8_t* spill;         // the caller's spill arena (tpz_columns)
  uint64_t spill_cap;
  uint64_t* spill_off;
  uint64_t* spill_used;   // zeroed before the launch
  uint32_t* bw_list;      // workspace: n_blocks entries (blocks for the bigwave kernel)
  uint32_t* bw_count;     // tail + kTailBw
  const uint32_t* rep;    // replicated slice-by-4 tables (the bigwave phase's CRC)
  const uint64_t* efirst; // exact ends layout (tpz_columns.d_entry_first) or null
  // flat layout (tpz_decode_blocks_flat): key / value columns and the blocks' first key / value
  // byte in them; null: slotted (data)
  uint8_t* keys;
  uint8_t* vals;
  const uint64_t* kfirst;
  const uint64_t* vfirst;
  uint32_t* tail;         // workspace: kTailCounters, zero at the launch (the tail kernel
                          // leaves them zero)
};
// Pair index of block b's first {kend, vend}: the exact layout's d_entry_first[b], or the
// slotted tpz_entry_base.
__host__ __device__ inline uint64_t ends_base(const uint64_t* efirst, uint64_t ext_b, uint64_t b) {
  return efirst ? efirst[b] : entry_base(ext_b, b);
}

void launch_decode(const LaunchArgs& a, hipStream_t stream);

// The decode's worklist counters (tpz_decode.hip decode_tail_kernel): zero before a decode, and
// zeroed again by the tail kernel's last workgroup.
enum TailCounter : int {
  kTailBig = 0,        // big list length
  kTailSpill,          // spill list length
  kTailBw,             // bigwave list length
  kTailBigTicket,      // big blocks claimed
  kTailBigDone,        // big blocks finished
  kTailSpillTicket,    // spill blocks claimed
  kTailExit,           // tail-kernel workgroups finished
  kTailRow,            // wave path: rows of 16 blocks claimed (decode_wave_kernel)
  kTailCounters,
  // Sticky, past the counters the tail kernel zeroes: set when a tail workgroup's wait for the
  // big phase timed out (tpz_decode_check reports it and clears it)
  kTailError = kTailCounters,
  // Sticky: set when tpz_decompress_blocks gave an LZ4 block a range that is not its exact length
  // (claimed sizes, tpz_decompressed_sizes_claimed); tpz_decompress_check reports and clears it
  kTailCodecInexact,
  kTailWords
};
__device__ __forceinline__ uint32_t tail_load(const uint32_t* c) {
  return __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Every thread of the workgroup: wait until *done reaches n, then see what the finished blocks
// wrote. Workgroups only wait for blocks that running workgroups hold (tickets), so the wait
// ends; it is still bounded (about a second), so that a counting bug cannot hang the device.
// A wait that times out is not passed over: it sets the sticky error word (tpz_decode_check
// returns TPZ_ERR_INTERNAL) and returns false, and the caller skips what depended on it.
__device__ __forceinline__ bool tail_wait(const uint32_t* done, uint32_t n, uint32_t* err,
                                          uint32_t* flag) {
  if (threadIdx.x == 0) {
    uint32_t i = 0;
    for (; i < (1u << 22) && tail_load(done) < n; i++) __builtin_amdgcn_s_sleep(2);
#ifdef TPZ_ABL_TAILLATE
    const bool late = true;   // diagnostic build (tests/test_gpu_tail_check.py): every wait times out
#else
    const bool late = tail_load(done) < n;
#endif
    if (late) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = late ? 0u : 1u;
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return __builtin_amdgcn_readfirstlane(*flag) != 0;
}

// Long blocks with few entries (tpz_bigwave.hip): one wave per block, straight from HBM.
struct BigWaveLaunch {
  const uint8_t* src;
  const uint64_t* ext;
  uint64_t src_bytes;
  const uint32_t* rep;          // replicated slice-by-4 tables
  const uint32_t* crc_tables;   // the decode tables (small shifts, inverse table)
  const uint32_t* list;
  uint8_t* data;
  uint32_t* ends;
  uint32_t* count;
  uint8_t* status;
  uint32_t* crc;
  uint32_t* spill_list;
  uint32_t* spill_count;
  uint32_t* big_list;
  uint32_t* big_count;
  const uint64_t* efirst;
};
// Launched between the wave kernel and decode_tail_kernel; ctr = the decode's tail counters.
void launch_bigwave(const BigWaveLaunch& a, uint32_t* ctr, uint32_t grid, hipStream_t stream);

// The spill path (tpz_spill.hip, phase C of the tail kernel): blocks the LDS paths hand over,
// decoded into the arena.
struct SpillLaunch {
  const uint8_t* src;
  const uint64_t* ext;
  uint64_t src_bytes;
  const uint32_t* crc_tables;
  const uint32_t* list;
  uint8_t* spill;
  uint64_t spill_cap;
  uint64_t* spill_off;
  uint64_t* spill_used;
  uint32_t* count;
  uint8_t* status;
  uint32_t* crc;
  // flat layout (keys non-null): the spill path writes the block's ends to
  // ends[2 * efirst[b] ..], its keys to keys[kfirst[b] ..] and its values to vals[vfirst[b] ..];
  // its arena record holds only a BAD_ENTRY block's class bytes
  uint32_t* ends;
  const uint64_t* efirst;
  uint8_t* keys;
  uint8_t* vals;
  const uint64_t* kfirst;
  const uint64_t* vfirst;
};

struct CrcLaunch {
  const uint8_t* src;
  const uint64_t* ext;
  uint64_t src_bytes;
  uint32_t n_ranges;
  uint32_t trailer;       // 0 (plain ranges) or 4 (FileObject: BE u32 trailer after the CRC)
  const uint32_t* tables; // kRangeTables x 256
  const uint32_t* rep;    // kCrcRepWords
  uint32_t* acc;          // workspace: n_ranges, zeroed before the launch
  uint32_t* crc;
  uint8_t* status;        // null for plain ranges
  uint32_t num_cus;
  bool acc_only;          // leave R0 of every range's main part in acc (no finish kernel:
                          // tpz_flat.hip open_finish_kernel finishes the files' tails)
};

void launch_crc_ranges(const CrcLaunch& a, hipStream_t stream);

struct SeekLaunch {
  const uint8_t* fk;
  const uint64_t* fk_pos;
  uint32_t n_blocks;
  const uint64_t* ext;
  const uint8_t* data;
  const uint32_t* ends;
  const uint32_t* count;
  const uint8_t* bstatus;
  const uint8_t* spill;
  const uint64_t* spill_off;
  const uint8_t* q;
  const uint64_t* q_pos;
  uint32_t n_q;
  uint32_t* out_block;
  uint32_t* out_entry;
  uint8_t* out_status;
  uint8_t* out_valid;
  const uint64_t* efirst;
};
void launch_seek(const SeekLaunch& a, hipStream_t stream);

struct BloomLaunch {
  const uint8_t* filter;
  uint64_t filter_len;
  const uint8_t* q;
  const uint64_t* q_pos;
  uint32_t n_q;
  uint8_t* out;
};
void launch_bloom(const BloomLaunch& a, hipStream_t stream);

struct BloomBuildLaunch {
  const uint8_t* keys;
  const uint64_t* key_pos;
  uint32_t n_keys;
  uint32_t k;
  uint64_t limit;       // bits in the array: (filter_len - 1) * 8
  uint8_t* filter;      // zeroed bit array, 4-byte aligned, padded to whole words
  uint64_t filter_words;  // (filter_len + 3) / 4
  void* work;           // bloom_build_work_bytes() of device scratch (the partitioned build)
};
// Scratch for the partitioned build (0: the filter is too big for it and the atomic kernel runs).
uint64_t bloom_build_work_bytes(uint32_t n_keys, uint32_t k, uint64_t limit);
void launch_bloom_build(const BloomBuildLaunch& a, hipStream_t stream);

struct PackLaunch {
  const uint64_t* ext;
  uint32_t n_blocks;
  const uint32_t* ends;
  const uint32_t* count;
  const uint8_t* status;
  const uint8_t* spill;
  const uint64_t* spill_off;
  const uint64_t* first;
  uint32_t* dense;
  const uint64_t* efirst;
};
void launch_pack_ends(const PackLaunch& a, hipStream_t stream);
// d_first[i] = sum of the header n of blocks < i (tpz_entry_first); `part` = workspace of
// entry_first_parts(n_blocks) u64.
uint64_t entry_first_parts(uint32_t n_blocks);
// tpz_flat_layout (tpz_flat.hip): first = 3 x (n_blocks + 1) u64 (entries, key bytes, value
// bytes: exclusive prefixes, totals at [n_blocks]); `part` = flat_scan_parts_words(n_blocks) u64.
uint64_t flat_scan_parts_words(uint32_t n_blocks);
// In place: a[i] = sum of a[j < i], a[n] = the total (n + 1 u64; part = flat_scan_parts_words(n)
// / 3 u64 suffices).
void launch_scan_u64(uint64_t* a, uint32_t n, uint64_t* part, hipStream_t stream);
// tpz_compress_blocks (tpz_compress.hip): scratch bytes for the per-block slots; the snappy
// encode, the scan of the sizes into dst_ext and the packing into dst.
uint64_t compress_scratch_bytes(uint64_t src_bytes, uint32_t n_blocks);
void launch_compress(const uint8_t* src, const uint64_t* ext, uint64_t src_bytes, uint32_t n_blocks,
                     uint32_t codec, uint8_t* scratch, uint64_t* dst_ext, uint64_t* part, uint8_t* dst,
                     uint32_t num_cus, hipStream_t stream);
void launch_flat_layout(const uint8_t* src, const uint64_t* ext, uint64_t src_bytes,
                        uint32_t n_blocks, uint64_t* first, uint64_t* part, uint32_t num_cus,
                        hipStream_t stream);
// tpz_verify_files_flat_layout (tpz_flat.hip): the whole-file CRC of n_files SST files (data
// region = blocks fblock[f] .. fblock[f + 1] - 1, then the tail) and the flat reservations of
// their data blocks from one read of the blocks.
struct OpenLaunch {
  const uint8_t* src;
  const uint64_t* bext;
  uint64_t src_bytes;
  uint32_t n_blocks;
  const uint32_t* fblock;   // n_files + 1
  uint32_t n_files;
  const uint8_t* tsrc;      // the files' tails (meta, bloom, offsets, trailer)
  const uint64_t* text;
  uint64_t tail_bytes;
  uint64_t* first;        // 3 x (n_blocks + 1)
  uint64_t* part;         // workspace: flat_scan_parts_words(n_blocks) u64
  uint32_t* cb;           // workspace: n_blocks
  uint32_t* tacc;         // workspace: n_files, zeroed (the tails' main-part R0, crc_window_kernel)
  const uint32_t* rep;    // the replicated slice-by-4 tables (crc_window_kernel)
  const uint32_t* dtab;   // decode tables
  const uint32_t* rtab;   // range tables
  uint32_t* crc;
  uint8_t* status;
  uint32_t num_cus;
};
void launch_open_flat(const OpenLaunch& a, hipStream_t stream);
void launch_entry_first(const uint8_t* src, const uint64_t* ext, uint64_t src_bytes,
                        uint32_t n_blocks, uint64_t* first, uint64_t* part, hipStream_t stream);
// first[i] = exclusive prefix of count over decoded (OK / OK_SPILLED) blocks, first[n] = total.
void launch_count_prefix(const uint32_t* count, const uint8_t* status, uint32_t n,
                         uint64_t* first, hipStream_t stream);

struct CodecLaunch {
  const uint8_t* src;
  const uint64_t* ext;
  uint64_t src_bytes;
  uint32_t n_blocks;
  uint64_t* size;          // tpz_decompressed_sizes output
  uint8_t* dst;            // tpz_decompress_blocks output
  const uint64_t* dst_ext;
  uint8_t* status;
  uint32_t* defer_list;    // workspace: n_blocks entries
  uint32_t* defer_count;   // workspace: zeroed before the launch
  uint32_t num_cus;
  bool claimed;            // tpz_decompressed_sizes_claimed
  uint32_t* inexact;       // workspace: sticky, read and cleared by tpz_decompress_check
};

void launch_codec_sizes(const CodecLaunch& a, hipStream_t stream);
void launch_decompress(const CodecLaunch& a, hipStream_t stream);

// The write side (tpz_encode.hip): block cuts (phase 0: nx + info; phase 1: the chain) and the
// block encode.
struct PlanLaunch {
  int phase;
  const uint64_t* kpos;
  const uint64_t* vpos;
  uint32_t n;
  uint32_t block_size;
  uint32_t* nx;        // workspace: n + 2 (n / 2048 + 1) (nx, per-workgroup maxima and bad entries)
  uint32_t* info;      // {max nx (w), first bad entry, n_blocks}: written by the kernels
  uint32_t w;          // phase 1: an upper bound of info[0] (the tables' row capacity)
  uint32_t chunk;      // phase 1: entries per chunk (>= w)
  int* tab_a;          // phase 1 workspace: 2 x K x w
  int* tab_b;
  uint32_t* cnt;       // phase 1 workspace: K
  uint32_t* first;
  uint64_t* ext;
  uint32_t* n_blocks;  // workspace: one u32
};
hipError_t launch_plan(const PlanLaunch& a, hipStream_t stream);
constexpr uint32_t kPlanChunk = 2048;  // minimum entries per plan chunk
constexpr uint32_t kPlanNextPer = 4096; // entries per plan_next_kernel workgroup

struct EncodeLaunch {
  const uint8_t* keys;
  const uint64_t* kpos;
  uint64_t key_bytes;
  const uint8_t* vals;
  const uint64_t* vpos;
  uint64_t val_bytes;
  const uint32_t* first;
  const uint64_t* ext;
  uint32_t n_blocks;            // or its bound, when plan_info is set
  const uint32_t* plan_info;    // tpz_plan_blocks_async's d_info (block count on the device), or null
  const uint32_t* crc_tables;
  uint8_t* out;
  uint32_t* big_list;   // workspace: n_blocks
  uint32_t* big_count;  // workspace: one u32
  uint32_t num_cus;
};
hipError_t launch_encode(const EncodeLaunch& a, hipStream_t stream);

}  // namespace tpz
