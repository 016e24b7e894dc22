/*
 * tpz_gpu.h — C ABI of the MI355X (gfx950) SSTable block decode + checksum path.
 *
 * This is the drop-in boundary for topazdb's read hot path. The reference has no FFI (it is a
 * plain Rust API); each entry point below replaces the reference items it names, and
 * INTEGRATION.md shows the `extern "C"` binding a topazdb maintainer adds on the Rust side.
 *
 *   tpz_decode_blocks_host  the same from host memory: H2D, decode and D2H pipelined in the
 *                           library (SsTable::read_block + FileObject::read, table.rs:154-164,
 *                           file_object.rs:23-27)
 *   tpz_decode_blocks       SsTable::read_block (src/table.rs:154-164) batched over many
 *                           blocks -> Block::decode (src/block.rs:46-65) -> compress::decode
 *                           tag dispatch (src/block/compress.rs:95-113) -> checksum::
 *                           verify_checksum (src/checksum.rs:12-21) -> every
 *                           BlockIterator::seek_to materialised (src/block/iterator.rs:63-83)
 *   tpz_crc32_ranges        checksum::calculate_checksum (src/checksum.rs:6-10) over many ranges
 *   tpz_verify_files        FileObject::open's whole-file CRC (src/table/file_object.rs:57-78),
 *                           batched over SST file images (SsTable::open, src/table.rs:91-112)
 *   tpz_decompress_blocks   compress::decode's codec step: snappy (src/block/compress.rs:104-107)
 *                           and lz4 (:108-111) blocks to their Uncompress form
 *   tpz_format_block_error  the reference's error strings (checksum.rs:18-21, compress.rs:97,102)
 *   tpz_plan_blocks +       the write side for compaction output: SsTableBuilder::add +
 *   tpz_encode_blocks       block_build (src/table/builder.rs:49-85) over entries in HBM
 *
 * Plain pointers and sizes only. Pointers named d_* are device (HBM) pointers of the context's
 * device; h_* are host pointers. `stream` is a hipStream_t passed as void* (NULL = default).
 * Every call is asynchronous on `stream` unless it says otherwise; the library never frees
 * caller memory and holds no global mutable state (one context per device; many host threads
 * may share it, and decodes on different streams run concurrently: every stream gets its own
 * device workspace).
 */
#ifndef TPZ_GPU_H
#define TPZ_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- ABI version -------------------------------------------------------------------------
 * Bumped on every incompatible change of a status value, a struct layout or a record format:
 *   1  round 1: statuses 0..7 with 6 = OVERLAP, 7 = TOO_LARGE (device limits); 5-field columns
 *   2  6 = OK_SPILLED, 7 = SPILL_FULL, 8 = CODEC_ERROR; spill arena fields in tpz_columns
 *   3  9 = BAD_ENTRY (a CRC-valid block with out-of-range entries decodes, with per-entry
 *      classes in its spill record, instead of MALFORMED); MALFORMED is now only the block-level
 *      panic of Block::decode
 *   4  tpz_decode_blocks_host takes snappy / lz4 blocks (tpz_host_columns.h_dext, data_cap);
 *      the exact ends layout (tpz_columns.d_entry_first, tpz_table.d_entry_first)
 *   5  the flat layout: tpz_flat_layout + tpz_decode_blocks_flat (tpz_flat_columns); no
 *      existing struct or status changed
 *   6  claimed LZ4 sizes: tpz_decompressed_sizes_claimed, tpz_decompress_check, TPZ_ERR_SIZES;
 *      tpz_verify_blocks_host (the host pipeline's verdict without the column downloads, for
 *      Block views of the caller's bytes). Round 6, same ABI: tpz_decode_blocks_host /
 *      tpz_verify_blocks_host return TPZ_ERR_NOMEM only for a short caller buffer (an internal
 *      chunk overflow is TPZ_ERR_INTERNAL), and tpz_decode_check also fails for a wave path row
 *      claim that timed out or was overwritten; new entry point tpz_verify_files_flat_layout
 *      (open + flat layout from one read of the blocks)
 * A consumer compiled against one header checks tpz_abi_version() == TPZ_ABI_VERSION. */
#define TPZ_ABI_VERSION 6
int tpz_abi_version(void);

/* ---- API return codes ------------------------------------------------------------------- */
typedef enum {
  TPZ_SUCCESS = 0,
  TPZ_ERR_INVALID_ARG = -1, /* null pointer, inconsistent sizes                               */
  TPZ_ERR_HIP = -2,         /* a HIP runtime call failed (tpz_last_error has the text)        */
  TPZ_ERR_NO_DEVICE = -3,   /* no gfx950 device with that index                               */
  TPZ_ERR_NOMEM = -4,
  TPZ_ERR_INTERNAL = -5,    /* a device-side consistency check failed (tpz_decode_check)      */
  TPZ_ERR_SIZES = -6        /* claimed codec sizes were not exact (tpz_decompress_check)      */
} tpz_err;

/* ---- per-block outcome (written to columns.status[i]) ------------------------------------
 * Maps one-to-one onto what Block::decode + iterating every entry does in the reference. */
typedef enum {
  TPZ_BLOCK_OK = 0,                /* Ok(Block); all entries decoded                         */
  TPZ_BLOCK_EMPTY = 1,             /* Err("data is empty")          compress.rs:96-98        */
  TPZ_BLOCK_BAD_TAG = 2,           /* Err("invaild data")           compress.rs:102          */
  TPZ_BLOCK_UNSUPPORTED_CODEC = 3, /* tag 2 (snappy) / 3 (lz4) given to tpz_decode_blocks
                                      without the codec step (tpz_decompress_blocks) first    */
  TPZ_BLOCK_CHECKSUM_MISMATCH = 4, /* Err("checksum: expected E, actual A") checksum.rs:18-21 */
  TPZ_BLOCK_MALFORMED = 5,         /* CRC-valid, but Block::decode itself panics on it: the
                                      decompressed block is shorter than its CRC, or the payload
                                      is too short for n / the n offsets (block.rs:49-59)      */
  TPZ_BLOCK_OK_SPILLED = 6,        /* Ok(Block); all entries decoded, into the spill arena
                                      (tpz_columns.d_spill) instead of the block's slot: the
                                      decoded bytes do not fit the slot (entries that overlap or
                                      repeat, which iterator.rs:63-83 accepts: 6*n > len or
                                      value_start(K) + V > len + 2), or the block is too long
                                      for the LDS paths (longer than TPZ_LDS_BLOCK_BYTES with
                                      64+ entries, or longer than TPZ_BIGWAVE_BLOCK_BYTES).
                                      Same answer as TPZ_BLOCK_OK.                             */
  TPZ_BLOCK_SPILL_FULL = 7,        /* Ok(Block) in the reference, but the caller's spill arena
                                      was too small for this block's record:
                                      d_spill_off[i] = the bytes it needs. Decode again with
                                      spill_cap >= *d_spill_used.                               */
  TPZ_BLOCK_CODEC_ERROR = 8,       /* Err of the codec: snap's decompress_vec rejects the
                                      stream (compress.rs:104-107)                           */
  TPZ_BLOCK_BAD_ENTRY = 9          /* Ok(Block): Block::decode succeeds (block.rs:46-65 checks
                                      no entry), but at least one entry lies out of range, and
                                      BlockIterator panics when it reaches that entry
                                      (iterator.rs:74-82, :91-109). Decoded into the spill arena
                                      like OK_SPILLED, count[i] = n, with one class byte per
                                      entry in the record (tpz_entry_class, below), so that a
                                      reader fails exactly where the reference's iterator does:
                                      a scan stopped by an empty key before the bad entry, a seek
                                      whose bisection never touches it and SsTable::open's first
                                      and last entry all succeed.                              */
} tpz_block_status;

/* Per-entry class of a TPZ_BLOCK_BAD_ENTRY block (its spill record), in the reference's terms
 * for entry i at o = offsets[i] in data (L = data.len(), src/block/iterator.rs:74-82):
 *   OK         the entry reads whole: key and value are in the record
 *   BAD_VALUE  key readable (o + 2 + klen <= L), value not (o + 4 + klen + vlen > L): the key is
 *              in the record, the value is empty; seek_to(i) panics, while seek_to_key's
 *              bisection (which reads keys only, :95-98) may compare against the key
 *   BAD_KEY    o + 2 > L or o + 2 + klen > L: key and value empty; any read of entry i panics */
typedef enum {
  TPZ_ENTRY_OK = 0,
  TPZ_ENTRY_BAD_VALUE = 1,
  TPZ_ENTRY_BAD_KEY = 2
} tpz_entry_class;

/* The largest block the LDS decode paths stage whole (every block a block_size <= 64 KiB
 * BlockBuilder emits fits); longer blocks with 64 or more entries are decoded by the spill path,
 * straight from HBM. */
#define TPZ_LDS_BLOCK_BYTES 94192u
/* Longer blocks with fewer than 64 entries are decoded one wave per block straight from HBM
 * (the bigwave path, as OK) up to this length; past it by the spill path (OK_SPILLED). No block
 * length limit exists: the spill path decodes any length the extents can express. */
#define TPZ_BIGWAVE_BLOCK_BYTES 0x40000000u

/* ---- batch input -------------------------------------------------------------------------
 * Encoded blocks back to back in one device buffer (an SST data region [0, meta_off), or the
 * data regions of many SSTs concatenated). Block i is d_src[d_ext[i] .. d_ext[i+1]); d_ext has
 * n_blocks+1 entries and is non-decreasing. src_bytes = d_ext[n_blocks] (host copy). Blocks may
 * start at any byte offset; d_src itself must be 16-byte aligned for tpz_decode_blocks and the
 * codec step (hipMalloc returns 256-byte aligned memory; TPZ_ERR_INVALID_ARG otherwise). The
 * CRC entry points take any d_src. */
typedef struct {
  const uint8_t* d_src;
  const uint64_t* d_ext;
  uint32_t n_blocks;
  uint64_t src_bytes;
} tpz_batch;

/* ---- decoded columns (the "slotted" layout) ----------------------------------------------
 * No global prefix pass: every block owns a slot derived from its input extent, so blocks
 * decode independently (and shard across GPUs) with no cross-block communication. Every slot
 * starts on a 128-byte line and is written in whole lines (HBM3E then never sees a partial-line
 * write from two different workgroups).
 *   data  : block i's slot starts at s = tpz_slot_base(ext[i], i). It holds the block's key
 *           bytes (every entry's key, in entry order) at data[s .. s + K), K = the block's key
 *           bytes, then its value bytes from data[s + tpz_value_start(K)] on (K rounded up to
 *           16; the bytes in between are unspecified). One stream per block: the copy writes it
 *           with whole-wave stores, and a consumer moves one contiguous range per block.
 *   ends  : entry j of block i (j < count[i]) has its exclusive end offsets at ends[2*(e+j)]
 *           (key, relative to s) and ends[2*(e+j)+1] (value, relative to s + vs),
 *           e = tpz_entry_base(ext[i], i), K = ends[2*(e+count[i]-1)] (0 when count is 0),
 *           vs = tpz_value_start(K):
 *             key_j   = data[s +      (j ? ends[2(e+j-1)]   : 0) .. s +      ends[2(e+j)]]
 *             value_j = data[s + vs + (j ? ends[2(e+j-1)+1] : 0) .. s + vs + ends[2(e+j)+1]]
 *   count[i]  : entries in block i (n) for OK, OK_SPILLED, BAD_ENTRY and SPILL_FULL, else 0
 *   status[i] : tpz_block_status
 *   crc[i]    : CRC-32 the device computed over the payload (valid for OK, OK_SPILLED,
 *               BAD_ENTRY, SPILL_FULL, MALFORMED (n / offsets too short), CHECKSUM_MISMATCH;
 *               the stored one is the payload's trailing u32)
 * Bytes of a slot beyond the block's own data are unspecified. A slot spans at most
 * len + 129 bytes (len = the block's encoded length), which never reaches the next slot.
 *
 * Spill arena. A block whose decoded bytes do not fit its slot (the reference iterator accepts
 * offsets that overlap or repeat, so n entries may materialise up to n * 65535 key and value
 * bytes each), one too long for the LDS paths, or one with out-of-range entries is decoded into
 * the caller's spill arena and reported TPZ_BLOCK_OK_SPILLED (TPZ_BLOCK_BAD_ENTRY for the last
 * kind). Its record starts at r = d_spill_off[i] (128-aligned):
 *   u32 ends[2*count[i]] at d_spill[r ..]         {kend, vend} pairs, exactly as in the slot
 *   stream at d_spill[r + tpz_spill_stream(count[i]) ..]: keys, then values from
 *                                                 tpz_value_start(K), as in the slot
 *   BAD_ENTRY only: count[i] class bytes (tpz_entry_class) at
 *                   d_spill[r + tpz_spill_classes(count[i], K, V) ..], K / V = the last kend /
 *                   vend; an entry's unreadable key or value is empty in ends and stream
 * (K and V each fit in 32 bits: at most 65535 entries of at most 65535 bytes.) Records are
 * placed by an atomic cursor; *d_spill_used = the bytes every spilled block of the call asked
 * for (the library zeroes it first). A record that does not fit spill_cap leaves the block
 * TPZ_BLOCK_SPILL_FULL with d_spill_off[i] = its size: decode the batch again with
 * spill_cap >= *d_spill_used. Batches written by topazdb's BlockBuilder with block_size <= 64 KiB
 * never spill; d_spill may then be NULL with spill_cap 0. */
typedef struct {
  uint8_t* d_data;          /* capacity tpz_data_capacity(src_bytes, n_blocks) bytes        */
  uint32_t* d_ends;         /* capacity 2 * tpz_entry_capacity(src_bytes, n_blocks) u32      */
  uint32_t* d_count;        /* n_blocks */
  uint8_t* d_status;        /* n_blocks */
  uint32_t* d_crc;          /* n_blocks */
  uint8_t* d_spill;         /* spill arena (see above), spill_cap bytes; may be NULL if 0   */
  uint64_t spill_cap;
  uint64_t* d_spill_off;    /* n_blocks: written for OK_SPILLED, BAD_ENTRY, SPILL_FULL only   */
  uint64_t* d_spill_used;   /* one u64                                                      */
  const uint64_t* d_entry_first; /* NULL: the slotted ends (tpz_entry_base). Else the exact
                                    ends layout: block i's {kend, vend} pairs at
                                    d_ends[2*d_entry_first[i] ..], d_ends holding
                                    2*d_entry_first[n_blocks] u32, d_entry_first from
                                    tpz_entry_first (see below)                             */
} tpz_columns;

/* Offset of a spilled record's stream from the record start: its 2*n u32 ends, 128-aligned. */
static inline uint64_t tpz_spill_stream(uint64_t n) {
  return (8u * n + 127u) & ~(uint64_t)127u;
}
/* Bytes of a spilled record with n entries, K key and V value bytes (128-aligned). */
static inline uint64_t tpz_spill_record_bytes(uint64_t n, uint64_t k, uint64_t v) {
  return tpz_spill_stream(n) + ((((k + 15u) & ~(uint64_t)15u) + v + 127u) & ~(uint64_t)127u);
}
/* Offset of a BAD_ENTRY record's class bytes from the record start (its ends and stream come
 * first); the record then spans tpz_spill_classes(n, K, V) + n bytes, 128-aligned. */
static inline uint64_t tpz_spill_classes(uint64_t n, uint64_t k, uint64_t v) {
  return tpz_spill_record_bytes(n, k, v);
}

static inline uint64_t tpz_slot_base(uint64_t ext_i, uint64_t i) {
  return ((ext_i + 127u) & ~(uint64_t)127u) + 256u * i;
}
static inline uint64_t tpz_value_start(uint64_t key_bytes) {
  return (key_bytes + 15u) & ~(uint64_t)15u;
}
static inline uint64_t tpz_entry_base(uint64_t ext_i, uint64_t i) {
  return 16u * (ext_i / 96u + i);
}
static inline uint64_t tpz_data_capacity(uint64_t src_bytes, uint64_t n_blocks) {
  return tpz_slot_base(src_bytes, n_blocks) + 128u;
}
static inline uint64_t tpz_entry_capacity(uint64_t src_bytes, uint64_t n_blocks) {
  return tpz_entry_base(src_bytes, n_blocks) + 16u;
}

/* Exported copies of the layout helpers for FFI callers that cannot use static inline. */
uint64_t tpz_layout_slot_base(uint64_t ext_i, uint64_t i);
uint64_t tpz_layout_value_start(uint64_t key_bytes);
uint64_t tpz_layout_entry_base(uint64_t ext_i, uint64_t i);
uint64_t tpz_layout_data_capacity(uint64_t src_bytes, uint64_t n_blocks);
uint64_t tpz_layout_entry_capacity(uint64_t src_bytes, uint64_t n_blocks);
uint64_t tpz_layout_spill_stream(uint64_t n);
uint64_t tpz_layout_spill_classes(uint64_t n, uint64_t k, uint64_t v);

/* ---- context ------------------------------------------------------------------------------ */
typedef struct tpz_ctx tpz_ctx;

/* Creates a context on HIP device `device` (uploads the CRC tables, sizes the launch grid for
 * the device's CU count). Fails with TPZ_ERR_NO_DEVICE unless the device is gfx950. */
tpz_err tpz_ctx_create(int device, tpz_ctx** out);
void tpz_ctx_destroy(tpz_ctx* ctx);

/* Pre-sizes the device workspace `stream` uses for batches of up to max_blocks blocks, so that
 * tpz_decode_blocks on that stream never allocates (needed before capturing it in a hipGraph).
 * Each stream gets its own workspace, so decodes on different streams may run concurrently.
 * Every call on one stream reuses that stream's workspace (worklists, plan buffers and the
 * pinned word tpz_plan_blocks reads back): calls that share a stream must not be made from
 * several host threads at once. Give each host thread its own stream. */
tpz_err tpz_ctx_reserve(tpz_ctx* ctx, uint32_t max_blocks, void* stream);

/* ---- the hot path ------------------------------------------------------------------------ */
/* Checksum-verify and decode every block of `batch` into `out`. Asynchronous on `stream`;
 * per-block outcomes land in out->d_status (no host sync, no host-visible error for a bad
 * block: that is data, not an API failure). */
tpz_err tpz_decode_blocks(tpz_ctx* ctx, const tpz_batch* batch, const tpz_columns* out,
                          void* stream);

/* Synchronizes `stream` and reports whether every decode on it so far ran to completion:
 * TPZ_ERR_INTERNAL (and the flag cleared) when a tail workgroup's bounded wait for the big
 * path timed out, so that blocks of the spill worklist may have been left undecoded (their
 * status/count/crc are then unspecified). The wait only times out if the device stalls for
 * about a second. The flag is sticky per stream: it covers every decode queued on `stream`
 * since the previous check, so a device-resident integration calls this once per batch (after
 * the batch's decode, before it trusts the outputs; tpz_decode_blocks_host and the Python layer
 * do). The flag is read and cleared in stream order (no null-stream copy). */
tpz_err tpz_decode_check(tpz_ctx* ctx, void* stream);

/* The exact ends layout. The slotted ends reserve the worst case (a pair per 6 input bytes,
 * ~1.36x the input in ends alone for 4 KiB blocks) so that blocks need no prefix pass; a caller
 * that keeps the decoded columns resident (a block cache in HBM) can instead reserve exactly n
 * pairs per block, 8 bytes per entry: d_first[i] = the sum over blocks 0..i-1 of the header n
 * (u16 at the block's first two bytes) of each block the decode parses in place (last byte 1,
 * len >= 7 + 2n, 6n <= len; 0 for any other block, whose pairs, if any, live in its spill
 * record), d_first[n_blocks] = the total, computed on the device (a header pass and a scan, no
 * host sync). A block that decodes in place has count == its header n, so its pairs fit. Pass
 * d_first as tpz_columns.d_entry_first / tpz_table.d_entry_first. The batch must be the one
 * the decode runs over (after the codec step). Asynchronous on `stream`; uses the stream's
 * workspace. */
tpz_err tpz_entry_first(tpz_ctx* ctx, const tpz_batch* batch, uint64_t* d_first, void* stream);

/* Dense entry ends for consumers that copy a batch out (e.g. back to the host): the slotted
 * ends reserve the worst case (a pair per 6 input bytes, ~1.33x the input) so that blocks need no
 * prefix pass; this packs the used pairs. d_first = exclusive prefix sums of out->d_count
 * (n_blocks + 1 entries, from the caller's device scan); block i's count[i] {kend, vend} pairs go
 * to d_dense[2*d_first[i] .. 2*d_first[i+1]) (for OK_SPILLED and BAD_ENTRY blocks from their
 * spill records; zeros for a block whose status is none of OK, OK_SPILLED, BAD_ENTRY). */
tpz_err tpz_pack_ends(tpz_ctx* ctx, const tpz_batch* batch, const tpz_columns* cols,
                      const uint64_t* d_first, uint32_t* d_dense, void* stream);

/* ---- the flat layout ---------------------------------------------------------------------
 * One dense key column and one dense value column for the whole batch: every key of every
 * block, in SsTableIterator order (blocks in batch order, entries in block order: what
 * BlockIterator::key() returns for each entry, src/block/iterator.rs:63-83), back to back, and
 * likewise every value; the {kend, vend} pairs give each entry's end within its block's run.
 *
 * tpz_flat_layout sizes the columns on the device (one pass over the batch and three scans, no
 * host sync): d_first holds 3 * (n_blocks + 1) u64, with st = n_blocks + 1:
 *   d_first[i]          entries of blocks 0..i-1 (the exact ends layout's d_entry_first)
 *   d_first[st + i]     key bytes of blocks 0..i-1: block i's keys start at d_keys[d_first[st + i]]
 *   d_first[2 st + i]   value bytes of blocks 0..i-1, likewise in d_values
 * and the totals at i = n_blocks (read them back to size the columns). A block's reservation is
 * what decoding it yields when its CRC matches: its header n entries and the bytes of every key
 * and value that reads whole (src/block/iterator.rs:74-82: an unreadable key or value reserves
 * nothing, as in TPZ_BLOCK_BAD_ENTRY), for a block with tag 1 and len >= 7 + 2n; nothing for any
 * other block (EMPTY, BAD_TAG, UNSUPPORTED_CODEC, MALFORMED). Run the codec step first for
 * snappy / lz4 batches. Asynchronous on `stream`; uses the stream's workspace. */
tpz_err tpz_flat_layout(tpz_ctx* ctx, const tpz_batch* batch, uint64_t* d_first, void* stream);

/* tpz_decode_blocks_flat: tpz_decode_blocks into the flat layout. Per block i (st as above):
 *   keys:   key_j   = d_keys  [kb + (j ? ends[2(e+j-1)]   : 0) .. kb + ends[2(e+j)]]
 *   values: value_j = d_values[vb + (j ? ends[2(e+j-1)+1] : 0) .. vb + ends[2(e+j)+1]]
 *   with e = d_first[i], kb = d_first[st + i], vb = d_first[2 st + i], j < count[i]
 *   d_count, d_status, d_crc: as tpz_columns. Every decoded block reports TPZ_BLOCK_OK or
 *   TPZ_BLOCK_BAD_ENTRY (no OK_SPILLED: the spill path writes the columns too); a block that
 *   fails its CRC keeps its reserved bytes, unspecified.
 *   d_spill / spill_cap / d_spill_off / d_spill_used: a BAD_ENTRY block's count[i] class bytes
 *   (tpz_entry_class) at d_spill[d_spill_off[i] ..] (records of n bytes rounded up to 128; the
 *   entry's unreadable key or value is empty in the columns), SPILL_FULL as in tpz_columns.
 *   May be NULL / 0 for batches without bad entries.
 * d_keys and d_values must be 16-byte aligned, with d_first[st + n_blocks] and
 * d_first[2 st + n_blocks] bytes; d_ends 2 * d_first[n_blocks] u32. Blocks share 16-byte chunks
 * of the columns at their boundaries: the decode writes those chunks byte-exactly (each block
 * its own bytes), so blocks still decode independently. Asynchronous on `stream`. */
typedef struct {
  uint8_t* d_keys;
  uint8_t* d_values;
  uint32_t* d_ends;
  const uint64_t* d_first;  /* from tpz_flat_layout over the same batch */
  uint32_t* d_count;
  uint8_t* d_status;
  uint32_t* d_crc;
  uint8_t* d_spill;
  uint64_t spill_cap;
  uint64_t* d_spill_off;
  uint64_t* d_spill_used;
} tpz_flat_columns;

tpz_err tpz_decode_blocks_flat(tpz_ctx* ctx, const tpz_batch* batch, const tpz_flat_columns* out,
                               void* stream);

/* ---- the host pipeline -------------------------------------------------------------------
 * SsTable::read_block for a whole run of blocks that sit in HOST memory (src/table.rs:154-164;
 * the bytes FileObject::read's pread returns, src/table/file_object.rs:23-27): the library
 * copies the blocks to the device in chunks, runs compress::decode's codec step on them where a
 * block is snappy or lz4 (src/block/compress.rs:104-111; topazdb's default codec is snappy,
 * src/opt.rs:48), decodes them (tpz_decode_blocks), packs the used entry ends (tpz_pack_ends)
 * and copies every output back, on three streams (upload, decode, download) so that both PCIe
 * directions stay busy. Synchronous: returns when every output is in host memory. The caller's
 * buffers are page-locked for the duration of the call when they are not already
 * (hipHostRegister); pinned buffers (hipHostMalloc) avoid that cost.
 *
 * Block i = h_src[h_ext[i] .. h_ext[i+1]) (h_ext non-decreasing, any alignment, any mix of
 * codec tags). The decoded layout is that of tpz_columns over the DECODED extents h_dext: for
 * a batch of Uncompress blocks h_dext = h_ext; when any block is snappy or lz4, h_dext[i+1] -
 * h_dext[i] = the block's length after the codec step (its Uncompress form; the codec's Err
 * leaves a 1-byte stub, tpz_decompressed_sizes), computed on the device chunk by chunk with no
 * whole-batch host sync. Outputs:
 *   h_data    data_cap bytes (0 = tpz_data_capacity(h_ext[n], n), enough for Uncompress
 *             batches; for snappy / lz4 blocks use tpz_data_capacity(bound, n) with bound from
 *             tpz_host_decoded_bound): the slotted stream layout, block i's slot at
 *             tpz_slot_base(h_dext[i], i)
 *   h_dext    n + 1 decoded extents (may be NULL for a batch without snappy / lz4 blocks)
 *   h_ends    every decoded block's {kend, vend} pairs, dense in block order: block i's at
 *             h_ends[2*h_first[i] ..]; ends_cap = its capacity in u32
 *   h_first   n + 1 entries: h_first[i] = pairs before block i (OK, OK_SPILLED and BAD_ENTRY
 *             blocks only)
 *   h_count, h_status, h_crc    n each, as tpz_columns; a block whose codec step failed has
 *             status TPZ_BLOCK_CODEC_ERROR (the reference's Err of the codec), count 0
 *   h_spill, spill_cap, h_spill_off, h_spill_used   as tpz_columns, in host memory: spilled
 *             blocks' records (the library's device arenas grow as needed)
 * Returns TPZ_ERR_NOMEM when ends_cap, spill_cap or data_cap is too small: h_first[n],
 * *h_spill_used and h_dext[n] then hold the sizes needed (the call can be repeated with larger
 * buffers; NOMEM has no other cause, so a repeat with buffers of those sizes succeeds). chunk_blocks = 0 picks the default (8,192 blocks per chunk: 34 MB of 4 KiB blocks,
 * the fastest of 4K..64K on MI355X, profiles/r2/e2e_sweep.jsonl). The streams and device buffers
 * of a call are kept by the context and reused by its next calls (one set per concurrent
 * caller). */
typedef struct {
  uint8_t* h_data;
  uint32_t* h_ends;
  uint64_t ends_cap;
  uint64_t* h_first;
  uint32_t* h_count;
  uint8_t* h_status;
  uint32_t* h_crc;
  uint8_t* h_spill;
  uint64_t spill_cap;
  uint64_t* h_spill_off;
  uint64_t* h_spill_used;
  uint64_t* h_dext;         /* n + 1 decoded extents, or NULL (see above)                   */
  uint64_t data_cap;        /* bytes at h_data; 0 = tpz_data_capacity(h_ext[n], n)          */
} tpz_host_columns;

/* An upper bound of h_dext[n] for blocks in host memory, from their headers alone: a snappy
 * block's preamble length + 1, an lz4 block's size prefix + 1 (lz4::block::decompress may keep
 * fewer bytes), any other block's own length. Size h_data with tpz_data_capacity(bound, n). */
tpz_err tpz_host_decoded_bound(const uint8_t* h_src, const uint64_t* h_ext, uint32_t n_blocks,
                               uint64_t* bound);

tpz_err tpz_decode_blocks_host(tpz_ctx* ctx, const uint8_t* h_src, const uint64_t* h_ext,
                               uint32_t n_blocks, const tpz_host_columns* out,
                               uint32_t chunk_blocks);

/* SsTable::read_block's checks for a run of blocks in host memory, with the decoded columns left
 * on the device: the reference's Block is {data: payload[2 + 2n ..], offsets} of the block's
 * Uncompress form (src/block.rs:46-65), so a host that holds the block bytes needs only the
 * device's verdict (CRC, tag, header) and, for snappy / lz4 blocks, the decompressed bytes to
 * build it without a copy (rust/topazdb-gpu/src/table/gpu.rs, read_blocks_gpu). Same pipeline as
 * tpz_decode_blocks_host (chunked H2D, codec step, decode) without the slot, ends and spill
 * downloads. Outputs: h_status, h_crc, h_count (n each, as tpz_host_columns); h_dext (n + 1, may
 * be NULL for a batch without snappy / lz4 blocks; h_ext is then the decoded layout); h_plain /
 * plain_cap: for a batch with snappy / lz4 blocks, h_dext[n] bytes receiving every block's
 * Uncompress form at h_dext[i] (tpz_host_decoded_bound bounds it); unused (may be NULL)
 * otherwise. Returns TPZ_ERR_NOMEM when plain_cap < h_dext[n] (h_dext[n] then holds the size
 * needed). */
tpz_err tpz_verify_blocks_host(tpz_ctx* ctx, const uint8_t* h_src, const uint64_t* h_ext,
                               uint32_t n_blocks, uint8_t* h_status, uint32_t* h_crc,
                               uint32_t* h_count, uint8_t* h_plain, uint64_t plain_cap,
                               uint64_t* h_dext, uint32_t chunk_blocks);

/* ---- whole-range CRC-32 ------------------------------------------------------------------
 * Ranges use the batch type: range i is d_src[d_ext[i] .. d_ext[i+1]) (d_ext non-decreasing,
 * n_blocks = number of ranges, src_bytes = d_ext[n]). Each range may be up to 2^35 bytes.
 *
 * checksum::calculate_checksum (src/checksum.rs:6-10) of every range: d_crc[i] = CRC-32/ISO-HDLC
 * of range i. Asynchronous on `stream`. */
tpz_err tpz_crc32_ranges(tpz_ctx* ctx, const tpz_batch* ranges, uint32_t* d_crc, void* stream);

/* FileObject::open's whole-file check (src/table/file_object.rs:57-78) for SST file images in
 * HBM: range i is a whole file; its CRC-32 over all but the last 4 bytes goes to d_crc[i] and
 * is compared with the big-endian u32 in those 4 bytes. d_status[i] = TPZ_BLOCK_OK,
 * TPZ_BLOCK_CHECKSUM_MISMATCH ("checksum: expected E, actual A", checksum.rs:18-21, with
 * A = d_crc[i]) or TPZ_BLOCK_MALFORMED (file shorter than 4 bytes: the reference's
 * `buf[size - CHECKSUM_SIZE..]` panics). Asynchronous on `stream`. */
tpz_err tpz_verify_files(tpz_ctx* ctx, const tpz_batch* files, uint32_t* d_crc,
                         uint8_t* d_status, void* stream);

/* SsTable::open for every file + tpz_flat_layout of their data blocks, from ONE read of the
 * blocks (the reference's open reads every byte for FileObject::open's CRC, src/table.rs:91-112,
 * src/table/file_object.rs:57-78, before the blocks are read again to decode them): the outputs of
 * tpz_verify_files over the files and of tpz_flat_layout(blocks, d_first).
 *   blocks : every file's data region (its blocks, [0, meta offset) of an SST), the files' regions
 *            back to back: the batch tpz_decode_blocks_flat then decodes
 *   d_file_block : n_files + 1 u32; file f's blocks are blocks d_file_block[f] ..
 *            d_file_block[f + 1] - 1 (d_file_block[n_files] = n_blocks)
 *   tails  : n_files ranges; tail f = the rest of file f after its data region (meta block,
 *            bloom filter, offsets and the 4-byte CRC trailer), so that file f is its data region
 *            followed by tail f. Each tail holds at least the trailer (a file whose tail is
 *            shorter than 4 bytes reports TPZ_BLOCK_MALFORMED with crc 0, as a file shorter than
 *            its trailer does in tpz_verify_files)
 *   d_crc, d_status : n_files, as tpz_verify_files
 * Both d_src 16-byte aligned. Asynchronous on `stream`; uses the stream's workspace. */
tpz_err tpz_verify_files_flat_layout(tpz_ctx* ctx, const tpz_batch* blocks,
                                     const uint32_t* d_file_block, const tpz_batch* tails,
                                     uint32_t* d_crc, uint8_t* d_status, uint64_t* d_first,
                                     void* stream);

/* ---- codec step of compress::decode (src/block/compress.rs:95-113) ------------------------
 * Snappy (tag 2) and LZ4 (tag 3) blocks are decompressed on the device into their Uncompress
 * (tag 1) form, so tpz_decode_blocks then verifies and decodes them like any block:
 *   1. tpz_decompressed_sizes: d_size[i] = the length block i has once decompressed and
 *      re-tagged: for tag 2 the snappy preamble's length + 1 (0 if the preamble is invalid);
 *      for tag 3 the length LZ4_decompress_safe decodes + 1 (lz4::block::decompress keeps only
 *      the decoded bytes, which may be fewer than the size prefix; 1 for an Err); the block's
 *      own length for any other block. No size limit: blocks past the LDS windows are
 *      decompressed straight from HBM to HBM.
 *   2. the caller forms d_dst_ext = exclusive prefix sums of d_size (n_blocks + 1 entries) and
 *      allocates d_dst (d_dst_ext[n] bytes).
 *   3. tpz_decompress_blocks writes block i's uncompressed form to d_dst[d_dst_ext[i] ..
 *      d_dst_ext[i+1]) (other tags are copied unchanged) and d_status[i] = TPZ_BLOCK_OK,
 *      or TPZ_BLOCK_CODEC_ERROR (the codec's Err). A failed block's range
 *      ends in tag 0, so decoding it reports BAD_TAG; its d_status is the reference's outcome.
 *   4. tpz_decode_blocks over (d_dst, d_dst_ext).
 * LZ4 acceptance is liblz4 1.9.3's LZ4_decompress_safe (the library the reference's lz4 crate
 * binds; restated in oracle/tpz_lz4.c and pinned against liblz4 in tests/test_lz4_oracle.py). */
tpz_err tpz_decompressed_sizes(tpz_ctx* ctx, const tpz_batch* batch, uint64_t* d_size,
                               void* stream);
/* Step 1 without LZ4's walk: a tag-3 block reports its size prefix + 1 (what
 * lz4::block::decompress allocates, compress.rs:108-111; the exact length of every stream
 * lz4::block::compress writes) instead of the length its stream decodes to; the exact walk only
 * where the prefix is invalid or larger than any stream of that length can decode to. Every other
 * block as tpz_decompressed_sizes. A stream that then decodes to another length or fails sets a
 * sticky word of the stream's workspace in tpz_decompress_blocks (that block's output is
 * CODEC_ERROR, the layout is not the exact one): tpz_decompress_check reports it, and the caller
 * sizes the batch with tpz_decompressed_sizes and decompresses it again. Asynchronous on
 * `stream`. */
tpz_err tpz_decompressed_sizes_claimed(tpz_ctx* ctx, const tpz_batch* batch, uint64_t* d_size,
                                       void* stream);
/* Synchronizes `stream`; TPZ_ERR_SIZES (and the word cleared) when a tpz_decompress_blocks on it
 * since the previous check ran over claimed sizes that were not exact, TPZ_SUCCESS otherwise. */
tpz_err tpz_decompress_check(tpz_ctx* ctx, void* stream);
tpz_err tpz_decompress_blocks(tpz_ctx* ctx, const tpz_batch* batch, uint8_t* d_dst,
                              const uint64_t* d_dst_ext, uint8_t* d_status, void* stream);

/* ---- batched point-get side ----------------------------------------
 * A table = its block metas' first keys plus the columns tpz_decode_blocks wrote for its
 * blocks (d_ext: the extents of the batch that decode ran over, i.e. after the codec step).
 *   tpz_seek_keys: for every query key, SsTableIterator::seek_to_key (src/table/iterator.rs:
 *     44-72): find_block_idx (src/table.rs:178-182, partition_point(first_key <= key) - 1,
 *     saturating; the lower-bound bisection), BlockIterator::seek_to_key in that block
 *     (src/block/iterator.rs:91-109: binary search, an equal key returns at once), then the
 *     next block's first entry when that iterator is invalid and a next block exists.
 *     d_block/d_entry = the position, d_valid = is_valid() (iterator.rs:50-52: the current key
 *     is non-empty), d_status = the status of the last block the seek read (non-OK: the
 *     reference's read_block_cached Err, or its panic for MALFORMED; a table with no blocks
 *     gives MALFORMED: block_metas[0] panics; so does a seek whose bisection reads the key of
 *     a BAD_KEY entry or which lands on a BAD_KEY / BAD_VALUE entry (iterator.rs:91-109, the
 *     reference's panic; entries of a BAD_ENTRY block the seek does not touch do not matter);
 *     OK_SPILLED and BAD_ENTRY blocks are read from their spill
 *     records and report OK).
 *   tpz_bloom_may_contain: SsTable::may_contain (src/table.rs:114-119) = Bloom::may_contain
 *     (src/bloom.rs:72-84) of xxh3_64(key) for every key; d_filter = Bloom::encode (the bit
 *     array, then k). d_out = 1 (may contain), 0 (absent), 2 (the reference panics: an empty
 *     filter, or no bit array with k > 0).
 * Keys are packed: key i = d_keys[d_key_pos[i] .. d_key_pos[i+1]). */
typedef struct {
  const uint8_t* d_first_keys;
  const uint64_t* d_first_pos; /* n_blocks + 1 */
  const uint64_t* d_ext;       /* n_blocks + 1 */
  uint32_t n_blocks;
  const uint8_t* d_data;
  const uint32_t* d_ends;
  const uint32_t* d_count;
  const uint8_t* d_status;
  const uint8_t* d_spill;      /* the decode's spill arena and record offsets (OK_SPILLED,
                                  BAD_ENTRY)                                               */
  const uint64_t* d_spill_off;
  const uint64_t* d_entry_first; /* the decode's tpz_columns.d_entry_first (NULL: slotted)   */
} tpz_table;

tpz_err tpz_seek_keys(tpz_ctx* ctx, const tpz_table* table, const uint8_t* d_keys,
                      const uint64_t* d_key_pos, uint32_t n_keys, uint32_t* d_block,
                      uint32_t* d_entry, uint8_t* d_status, uint8_t* d_valid, void* stream);
tpz_err tpz_bloom_may_contain(tpz_ctx* ctx, const uint8_t* d_filter, uint64_t filter_len,
                              const uint8_t* d_keys, const uint64_t* d_key_pos, uint32_t n_keys,
                              uint8_t* d_out, void* stream);
/* xxh3_64 (seed 0) on the host: the hash the reference's bloom uses (xxhash-rust 0.8.5). */
uint64_t tpz_host_xxh3_64(const uint8_t* h_buf, uint64_t len);

/* Bloom::from_keys (src/bloom.rs:48-70) for keys in HBM (SsTableBuilder::build_bloom,
 * src/table/builder.rs:132-141, over xxh3_64 of every added key):
 *   tpz_bloom_geometry (host): the filter's length in bytes (bit array + the k byte) and k for
 *     n_keys keys and false-positive rate fpp, with the reference's f64 arithmetic and saturating
 *     casts; TPZ_ERR_INVALID_ARG unless 0 <= fpp < 1 (bloom.rs:49 asserts).
 *   tpz_bloom_build: writes the filter (Bloom::encode) to d_filter[0 .. filter_len). d_filter must
 *     be 4-byte aligned with room for (filter_len + 3) & ~3 bytes. Asynchronous on `stream`;
 *     uses the stream's grow-only workspace (4 B per probe: n_keys * k * 4 bytes plus slice
 *     histograms), so one build at a time per stream, as with the other workspace users. */
tpz_err tpz_bloom_geometry(uint64_t n_keys, double fpp, uint64_t* filter_len, uint32_t* k);
tpz_err tpz_bloom_build(tpz_ctx* ctx, const uint8_t* d_keys, const uint64_t* d_key_pos,
                        uint32_t n_keys, double fpp, uint8_t* d_filter, void* stream);

/* ---- device write side (SURVEY.md §8f row 4's alternative: compaction output) ------------
 * A run of sorted entries in HBM becomes SST data-region blocks, byte for byte what
 * SsTableBuilder::add + block_build (src/table/builder.rs:49-85) writes with
 * CompressOptions::Uncompress: BlockBuilder's fill rule (src/block/builder.rs:26-41: an entry
 * joins the block while size + encode_len + 2 <= block_size), Block::encode (src/block.rs:31-44),
 * Entry::encode (builder.rs:72-81), the CRC (src/checksum.rs:6-10) and the tag
 * (src/block/compress.rs:85-89). Entry e: key = d_keys[d_kpos[e] .. d_kpos[e+1]), value =
 * d_vals[d_vpos[e] .. d_vpos[e+1]) (d_kpos/d_vpos: n_entries + 1 non-decreasing offsets; key_bytes
 * and val_bytes = the readable bytes at d_keys / d_vals, at least d_kpos[n] / d_vpos[n]).
 *   tpz_plan_blocks: the block cuts. d_first[b] = first entry of block b, d_ext[b] = its byte
 *     offset in the data region (SsTableBuilder's data.len() when it was built, i.e.
 *     BlockMeta::offset), for b <= n_blocks (d_first[n_blocks] = n_entries, d_ext[n_blocks] = the
 *     region's length); both need n_entries + 1 entries. SYNCHRONOUS on `stream` (it returns
 *     *h_n_blocks). An empty key (builder.rs:27 asserts) or an entry no block can hold (encode_len
 *     + 2 > block_size: SsTableBuilder::add recurses without end, table/builder.rs:57-60) makes it
 *     return TPZ_ERR_INVALID_ARG with *h_bad_entry = the first such entry (UINT64_MAX otherwise).
 *     block_size must be in (2, 65536]: past 64 KiB the reference's u16 offsets wrap.
 *   tpz_encode_blocks: writes block b to d_out[d_ext[b] .. d_ext[b+1]) (d_out 16-byte aligned,
 *     d_ext[n_blocks] bytes; no byte outside the blocks is written) for d_first / d_ext /
 *     n_blocks exactly as tpz_plan_blocks returned them for these entries and block_size.
 *     Asynchronous on `stream`; uses the stream's workspace (like tpz_decode_blocks).
 *   tpz_plan_blocks_async: tpz_plan_blocks with its results left on the device:
 *     d_info[0] = the most entries a block starting at any entry would take (>= the longest
 *     block; the plan's chunk tables are that wide), d_info[1] = the first entry the reference rejects
 *     (0xFFFFFFFF: none; d_first / d_ext are then meaningless), d_info[2] = n_blocks (4 u32 of
 *     device memory). No host round trip for block_size <= TPZ_PLAN_ASYNC_MAX_BLOCK (every block
 *     then holds at most 2048 entries, the transfer tables are sized from that bound); a larger
 *     block size reads the longest block back once (its plan chunks follow it). tpz_plan_blocks
 *     is this call plus one read of d_info.
 *   tpz_encode_blocks_async: tpz_encode_blocks with the block count read on the device from
 *     tpz_plan_blocks_async's d_info (a plan with a rejected entry encodes nothing). d_out needs
 *     d_ext[n_blocks] bytes; key_bytes + val_bytes + 13 * n_entries bounds that without reading it.
 * BlockMeta::first_key of block b is entry d_first[b]'s key. */
#define TPZ_PLAN_ASYNC_MAX_BLOCK 10242u
typedef struct {
  const uint8_t* d_keys;
  const uint64_t* d_kpos;
  const uint8_t* d_vals;
  const uint64_t* d_vpos;
  uint32_t n_entries;
  uint64_t key_bytes;
  uint64_t val_bytes;
} tpz_entries;

tpz_err tpz_plan_blocks(tpz_ctx* ctx, const tpz_entries* entries, uint32_t block_size,
                        uint32_t* d_first, uint64_t* d_ext, uint32_t* h_n_blocks,
                        uint64_t* h_bad_entry, void* stream);
tpz_err tpz_encode_blocks(tpz_ctx* ctx, const tpz_entries* entries, const uint32_t* d_first,
                          const uint64_t* d_ext, uint32_t n_blocks, uint8_t* d_out, void* stream);
tpz_err tpz_plan_blocks_async(tpz_ctx* ctx, const tpz_entries* entries, uint32_t block_size,
                              uint32_t* d_first, uint64_t* d_ext, uint32_t* d_info, void* stream);
tpz_err tpz_encode_blocks_async(tpz_ctx* ctx, const tpz_entries* entries, const uint32_t* d_first,
                                const uint64_t* d_ext, const uint32_t* d_info, uint8_t* d_out,
                                void* stream);

/* ---- host write side (inputs for benches and the table facade) ---------------------------
 * SsTableBuilder::add + block_build (src/table/builder.rs:49-85) with BlockBuilder's fill rule
 * (src/block/builder.rs:26-41) and Block::encode + Uncompress (src/block.rs:31-44,
 * src/block/compress.rs:85-89): packs entries e (key = keys[kpos[e]..kpos[e+1]), value likewise)
 * into blocks written back to back into h_out, block i = [ext[i], ext[i+1]). Host memory only.
 * Returns TPZ_ERR_INVALID_ARG for an empty key or an entry no block can hold, TPZ_ERR_NOMEM
 * when out_cap / ext_cap are too small. */
int tpz_build_blocks(const uint8_t* h_keys, const uint64_t* h_kpos, const uint8_t* h_vals,
                     const uint64_t* h_vpos, uint64_t n_entries, uint32_t block_size,
                     uint8_t* h_out, uint64_t out_cap, uint64_t* h_ext, uint64_t ext_cap,
                     uint64_t* n_blocks, uint64_t* out_len);
/* compress::encode with CompressOptions::Snappy (src/block/compress.rs:66-71) over a batch of
 * Uncompress blocks: every tag-1 block i = h_src[h_ext[i] .. h_ext[i+1]) is written to h_out as
 * snappy_raw(payload | crc) | 2, other blocks unchanged; h_out_ext gets n_blocks + 1 extents.
 * Host memory only; out_cap >= 32 * n_blocks + 2 * h_ext[n_blocks] always suffices. */
int tpz_snappy_encode_blocks(const uint8_t* h_src, const uint64_t* h_ext, uint64_t n_blocks,
                             uint8_t* h_out, uint64_t out_cap, uint64_t* h_out_ext,
                             uint64_t* out_len);
/* compress::encode with CompressOptions::Lz4 (src/block/compress.rs:73-77): every tag-1 block
 * becomes u32 LE size (payload | crc) | lz4_block(payload | crc) | 3 (lz4::block::compress with
 * prepend_size), other blocks unchanged. Host memory only; out_cap >= 32 * n_blocks +
 * 2 * h_ext[n_blocks] always suffices. */
int tpz_lz4_encode_blocks(const uint8_t* h_src, const uint64_t* h_ext, uint64_t n_blocks,
                          uint8_t* h_out, uint64_t out_cap, uint64_t* h_out_ext,
                          uint64_t* out_len);
/* ---- compaction output with a codec, on the device ---------------------------------------
 * compress::encode(data, opt) (src/block/compress.rs:66-77, :82-93) for every block of a batch
 * of Uncompress blocks in HBM (tpz_encode_blocks' output), opt = the SST's compress_option
 * (src/table/builder.rs:74; Snappy by default, src/opt.rs:48):
 *   codec 2 (Snappy): block i = payload | crc | 1 becomes snappy_raw(payload | crc) | 2
 *   codec 3 (Lz4):    u32 LE size | lz4_block(payload | crc) | 3 (lz4::block::compress with
 *                     prepend_size; every match ends 5 bytes and starts 12 bytes before the
 *                     end, as LZ4_decompress_safe requires)
 * written back to back into d_dst; d_dst_ext gets n_blocks + 1 extents (its last entry = the
 * bytes written), so BlockMeta::offset of block i is d_dst_ext[i] (src/table/builder.rs:74-84).
 * Blocks with another tag are copied unchanged; any other codec is TPZ_ERR_INVALID_ARG. The
 * streams decode with snap / liblz4 to exactly payload | crc; they are not byte-identical to
 * those libraries' encoders. Blocks whose payload is longer than 4,336 bytes (block_size past
 * 4 KiB) are emitted as literal elements only: valid streams, a few bytes larger than the
 * payload (the match finder works on blocks staged whole in LDS). d_dst needs
 * tpz_layout_compress_bound(src_bytes, n_blocks) bytes. batch->d_src and d_dst must be 16-byte
 * aligned (TPZ_ERR_INVALID_ARG otherwise). Asynchronous on `stream`; uses the stream's workspace
 * (scratch of that bound). */
uint64_t tpz_layout_compress_bound(uint64_t src_bytes, uint64_t n_blocks);
tpz_err tpz_compress_blocks(tpz_ctx* ctx, const tpz_batch* batch, uint32_t codec, uint8_t* d_dst,
                            uint64_t* d_dst_ext, void* stream);

/* CRC-32/ISO-HDLC on the host (checksum::calculate_checksum, src/checksum.rs:6-10). */
uint32_t tpz_host_crc32(const uint8_t* h_buf, uint64_t len);

/* ---- errors ------------------------------------------------------------------------------ */
/* Writes the reference's error text for a block outcome into buf (NUL-terminated):
 * "data is empty", "invaild data", "checksum: expected E, actual A" (decimal, as Rust's {}),
 * "unsupported codec", "malformed block", "spill arena too small", "decompression failed",
 * "" for OK, OK_SPILLED and BAD_ENTRY (an Ok(Block); its bad entries panic on access).
 * Returns the text length. */
int tpz_format_block_error(int status, uint32_t crc_expected, uint32_t crc_actual, char* buf,
                           size_t cap);
/* Last HIP error text seen by this thread (empty if none). */
const char* tpz_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* TPZ_GPU_H */
