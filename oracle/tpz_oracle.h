/*
 * tpz_oracle.h — CPU restatement of topazdb's SSTable block decode + checksum path.
 *
 * TEST INFRASTRUCTURE ONLY. This is the checker for the HIP path, not part of the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it
 * (oracle/liboracle.so). The product library (topazdb_amd/libtpz_gpu.so) never links it.
 *
 * Parity pinning: the reference is Rust and cannot be built here (no cargo), so
 * this restatement is pinned by (1) the reference's own generator-based known-answer tests
 * restated in tests/test_oracle.py, (2) CRC-32 known answers from zlib.crc32 and
 * (3) fixtures from an independent pure-Python restatement (tests/golden/make_golden.py).
 *
 * Every function cites the reference file:line it restates (paths relative to the reference).
 */
#ifndef TPZ_ORACLE_H
#define TPZ_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Per-block outcome; numbering is shared with include/tpz_gpu.h (tpz_block_status). */
enum {
  TPZO_OK = 0,          /* Block::decode Ok                                   */
  TPZO_EMPTY = 1,       /* Err("data is empty")      src/block/compress.rs:96-98 */
  TPZO_BAD_TAG = 2,     /* Err("invaild data")       src/block/compress.rs:102   */
  TPZO_UNSUPPORTED = 3, /* no longer produced: lz4 (tag 3) is decoded (tpz_lz4.c) */
  TPZO_CHECKSUM = 4,    /* Err("checksum: ...")      src/checksum.rs:12-21       */
  TPZO_MALFORMED = 5,   /* Block::decode itself panics   src/block.rs:49-59             */
  /* 6 (OK_SPILLED) and 7 (SPILL_FULL) are device-side placements of an Ok block (the spill
   * arena of include/tpz_gpu.h); the reference, and so this oracle, reports them TPZO_OK. */
  TPZO_CODEC = 8,       /* the codec returns Err: snap's decompress_vec (compress.rs:104-107),
                           lz4::block::decompress (compress.rs:108-111)                     */
  TPZO_BAD_ENTRY = 9    /* Block::decode is Ok (block.rs:46-65 checks no entry), but some entry
                           is out of range: BlockIterator panics when it reaches it
                           (iterator.rs:74-82); per-entry classes below                     */
};

/* Entry classes (tpz_entry_class of include/tpz_gpu.h): entry i at o = offsets[i], L = data.len():
 *   0 OK         reads whole                                     iterator.rs:74-82
 *   1 BAD_VALUE  o + 2 + klen <= L, but the value part panics    :80-82
 *   2 BAD_KEY    o + 2 > L or o + 2 + klen > L                    :74-78 (and :95-98) */
enum { TPZO_ENTRY_OK = 0, TPZO_ENTRY_BAD_VALUE = 1, TPZO_ENTRY_BAD_KEY = 2 };

/* Iterator return codes: 0, TPZO_ERR (read_block_cached returned Err), TPZO_PANIC (the
 * reference panics: an out-of-range entry read, or an assert). */
enum { TPZO_ERR = -1, TPZO_PANIC = -2 };

/* CRC-32/ISO-HDLC bit by bit (crc32fast's function): src/checksum.rs:6-10. */
uint32_t tpzo_crc32(const uint8_t* p, size_t n);

/* The same CRC via PCLMULQDQ folding (crc32fast's x86 algorithm); used by the CPU baseline. */
uint32_t tpzo_crc32_fast(const uint8_t* p, size_t n);

/* Count pass: entries / key bytes / value bytes the decode pass will emit. */
void tpzo_batch_sizes(const uint8_t* src, const uint64_t* ext, uint32_t n_blocks,
                      uint64_t* n_entries, uint64_t* key_bytes, uint64_t* val_bytes);

/* Block::decode (src/block.rs:46-65, snappy blocks decompressed first as compress.rs:104-107)
 * + BlockIterator::seek_to for every index (src/block/iterator.rs:63-83) over blocks
 * [ext[i], ext[i+1]). Dense outputs in block order:
 * entries are emitted for TPZO_OK and TPZO_BAD_ENTRY blocks (count = n); an entry's unreadable
 * key or value is empty and cls[e] (may be NULL) holds its class. crc_actual is the CRC the
 * reference computes over the payload (0 when it never gets that far). Returns 0. */
int tpzo_decode_batch(const uint8_t* src, const uint64_t* ext, uint32_t n_blocks,
                      uint8_t* status, uint32_t* crc_actual, uint32_t* crc_expected,
                      uint32_t* count, uint32_t* klen, uint32_t* vlen,
                      uint8_t* keys, uint8_t* vals, uint8_t* cls);

/* FileObject::open (src/table/file_object.rs:57-78) + SsTable::open (src/table.rs:75-112).
 * Verifies the whole-file CRC, walks the trailer chain and returns the data-block extents
 * (ext[0..n_blocks], last = meta_off, src/table.rs:154-161). Returns 0 on success,
 * -1 file checksum mismatch, -2 malformed trailer, -3 ext_cap too small. */
int tpzo_sst_parse(const uint8_t* file, size_t len, uint64_t* ext, uint32_t ext_cap,
                   uint32_t* n_blocks, uint64_t* meta_off, uint64_t* bloom_off);

/* ---- iterator restatement (src/block/iterator.rs, src/table/iterator.rs) ---------------- */
typedef struct tpzo_sst_iter tpzo_sst_iter;

/* SsTableIterator over an in-memory SST file image (the caller keeps `file` alive). */
tpzo_sst_iter* tpzo_sst_iter_create(const uint8_t* file, size_t len);
void tpzo_sst_iter_destroy(tpzo_sst_iter* it);
/* These return 0, TPZO_ERR or TPZO_PANIC. */
int tpzo_sst_iter_seek_to_first(tpzo_sst_iter* it);                      /* :18-42 */
int tpzo_sst_iter_seek_to_key(tpzo_sst_iter* it, const uint8_t* k, size_t kl); /* :44-72 */
int tpzo_sst_iter_next(tpzo_sst_iter* it);                               /* :88-95 */
int tpzo_sst_iter_is_valid(const tpzo_sst_iter* it);                     /* :84-86 */
const uint8_t* tpzo_sst_iter_key(const tpzo_sst_iter* it, size_t* len);
const uint8_t* tpzo_sst_iter_value(const tpzo_sst_iter* it, size_t* len);
uint32_t tpzo_sst_iter_block_idx(const tpzo_sst_iter* it);
/* SsTable::init_samllest_biggest_key (src/table.rs:143-151) over the iterator's table: read the
 * last block, seek_to_first, seek_to_last, assert is_valid. 0 (key and len = biggest_key),
 * TPZO_ERR or TPZO_PANIC. */
int tpzo_sst_biggest_key(tpzo_sst_iter* it, const uint8_t** key, size_t* len);

/* ---- snappy raw format (tpz_snappy.c; codec 2, src/block/compress.rs:66-71, 104-107) ------
 * decompress: 0 and *out_len on success, -1 where snap's decoder returns Err.
 * compress: a valid stream for fixtures (dst >= 64 + 2n); mode 0 = copy-1/copy-2,
 * 1 = copy-2 only, 2 = copy-4 only, 3 = literals only. */
int tpzo_snappy_uncompressed_len(const uint8_t* src, size_t n, uint64_t* len);
int tpzo_snappy_decompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap,
                           uint64_t* out_len);
size_t tpzo_snappy_compress(const uint8_t* src, size_t n, uint8_t* dst, int mode);

/* ---- LZ4 block format (tpz_lz4.c; codec 3, src/block/compress.rs:73-77, 108-111) --------
 * tpzo_lz4_decompress_safe: LZ4_decompress_safe as liblz4 1.9.3 accepts (out may be NULL:
 * validity and length only); returns the decoded length or -1.
 * tpzo_lz4_prefixed_size: lz4::block::decompress's size-prefix checks; 0 or -1.
 * tpzo_lz4_compress: a valid raw block (dst >= 16 + n + n / 255) for fixtures; mode 1 =
 * literals only. */
int64_t tpzo_lz4_decompress_safe(const uint8_t* in, int64_t src_size, uint8_t* out,
                                 int64_t out_size);
int tpzo_lz4_prefixed_size(const uint8_t* src, size_t n, int64_t* size);
size_t tpzo_lz4_compress(const uint8_t* src, size_t n, uint8_t* dst, int mode);

/* ---- CPU baseline: benches/sstable_iter_read.rs:60-79 restated --------------------------
 * SsTableIterator::create_and_seek_to_first + `while is_valid { next }` over SST files on
 * disk: one pread per block (file_object.rs:23-27), codec copy (compress.rs:103), CRC verify,
 * offsets Vec, and a malloc+memcpy per key and per value (iterator.rs:78,82). `paths` are
 * independent SSTs; `threads` workers each own whole files (Arc<SsTable> sharing in the
 * reference). Returns wall seconds for `iters` full passes; *bytes = encoded block bytes read
 * per pass, *entries = entries visited per pass. */
double tpzo_bench_iter_read(const char* const* paths, uint32_t n_paths, uint32_t threads,
                            uint32_t iters, uint64_t* bytes, uint64_t* entries);

/* ---- write side: SsTableBuilder's data region (Uncompress), the checker of the device encode
 * (builder.rs:26-81, table/builder.rs:49-85, block.rs:31-44). Returns n_blocks, -1 (capacity)
 * or -2 (*bad = an entry with an empty key or too large for any block). */
int64_t tpzo_build_blocks(const uint8_t* keys, const uint64_t* kpos, const uint8_t* vals,
                          const uint64_t* vpos, uint64_t n, uint32_t block_size, uint8_t* out,
                          uint64_t out_cap, uint64_t* ext, uint64_t* first, uint64_t ext_cap,
                          uint64_t* bad);

#ifdef __cplusplus
}
#endif
#endif
