/*
 * tpz_oracle.c — CPU restatement of topazdb's SSTable block decode + checksum path.
 * TEST INFRASTRUCTURE ONLY (see tpz_oracle.h): the checker and the CPU baseline, never the
 * product. Built by oracle/Makefile with gcc into oracle/liboracle.so.
 */
#define _GNU_SOURCE
#include "tpz_oracle.h"

#include <fcntl.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>
#include <immintrin.h>

/* bytes::Buf::get_u16 / get_u32 are big-endian (bytes crate; src/block.rs:51,54). */
static inline uint32_t be16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }
static inline uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

/* src/checksum.rs:6-10 — crc32fast::Hasher = CRC-32/ISO-HDLC: reflected polynomial
 * 0xEDB88320, init 0xFFFFFFFF, xorout 0xFFFFFFFF. Deliberately bit-serial (no tables) so it
 * shares nothing with the device's table-driven algorithm. */
uint32_t tpzo_crc32(const uint8_t* p, size_t n) {
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; i++) {
    c ^= p[i];
    for (int b = 0; b < 8; b++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
  }
  return c ^ 0xFFFFFFFFu;
}

/* ---- fast CRC for the CPU-baseline loop only ----------------------------------------------
 * crc32fast (the reference's dependency) runs a PCLMULQDQ folding kernel on x86; the baseline
 * must not be slowed by the checker's bit-serial CRC, so it uses the same published folding
 * algorithm (Gopal et al., "Fast CRC Computation for Generic Polynomials Using PCLMULQDQ",
 * constants for the reflected 0xEDB88320 polynomial) with a slicing-by-8 tail/fallback. */
static uint32_t s8[8][256];
static void s8_init(void) {
  if (s8[0][1]) return;
  for (uint32_t b = 0; b < 256; b++) {
    uint32_t c = b;
    for (int i = 0; i < 8; i++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    s8[0][b] = c;
  }
  for (int k = 1; k < 8; k++)
    for (uint32_t b = 0; b < 256; b++) s8[k][b] = (s8[k - 1][b] >> 8) ^ s8[0][s8[k - 1][b] & 0xFF];
}
/* raw update: register c (already inverted), returns register */
static uint32_t s8_update(uint32_t c, const uint8_t* p, size_t n) {
  while (n >= 8) {
    uint32_t lo, hi;
    memcpy(&lo, p, 4);
    memcpy(&hi, p + 4, 4);
    lo ^= c;
    c = s8[7][lo & 0xFF] ^ s8[6][(lo >> 8) & 0xFF] ^ s8[5][(lo >> 16) & 0xFF] ^ s8[4][lo >> 24] ^
        s8[3][hi & 0xFF] ^ s8[2][(hi >> 8) & 0xFF] ^ s8[1][(hi >> 16) & 0xFF] ^ s8[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) c = (c >> 8) ^ s8[0][(c ^ *p++) & 0xFF];
  return c;
}
__attribute__((target("pclmul,sse4.1")))
static __m128i fold128(__m128i a, __m128i b, __m128i k) {
  return _mm_xor_si128(_mm_xor_si128(b, _mm_clmulepi64_si128(a, k, 0x00)),
                       _mm_clmulepi64_si128(a, k, 0x11));
}
__attribute__((target("pclmul,sse4.1")))
static uint32_t clmul_crc(const uint8_t* p, size_t n) { /* n >= 64; returns final CRC */
  const __m128i k1k2 = _mm_set_epi64x(0x1c6e41596LL, 0x154442bd4LL);
  const __m128i k3k4 = _mm_set_epi64x(0x0ccaa009eLL, 0x1751997d0LL);
  const __m128i k5 = _mm_set_epi64x(0, 0x163cd6124LL);
  const __m128i pu = _mm_set_epi64x(0x1F7011641LL, 0x1DB710641LL);
  const __m128i m32 = _mm_set_epi32(0, 0, 0, -1);
  __m128i x3 = _mm_loadu_si128((const __m128i*)p), x2 = _mm_loadu_si128((const __m128i*)(p + 16));
  __m128i x1 = _mm_loadu_si128((const __m128i*)(p + 32)), x0 = _mm_loadu_si128((const __m128i*)(p + 48));
  x3 = _mm_xor_si128(x3, _mm_cvtsi32_si128((int)0xFFFFFFFF));
  p += 64;
  n -= 64;
  while (n >= 64) {
    x3 = fold128(x3, _mm_loadu_si128((const __m128i*)p), k1k2);
    x2 = fold128(x2, _mm_loadu_si128((const __m128i*)(p + 16)), k1k2);
    x1 = fold128(x1, _mm_loadu_si128((const __m128i*)(p + 32)), k1k2);
    x0 = fold128(x0, _mm_loadu_si128((const __m128i*)(p + 48)), k1k2);
    p += 64;
    n -= 64;
  }
  __m128i x = fold128(x3, x2, k3k4);
  x = fold128(x, x1, k3k4);
  x = fold128(x, x0, k3k4);
  while (n >= 16) {
    x = fold128(x, _mm_loadu_si128((const __m128i*)p), k3k4);
    p += 16;
    n -= 16;
  }
  x = _mm_xor_si128(_mm_clmulepi64_si128(x, k3k4, 0x10), _mm_srli_si128(x, 8));
  x = _mm_xor_si128(_mm_clmulepi64_si128(_mm_and_si128(x, m32), k5, 0x00), _mm_srli_si128(x, 4));
  __m128i t1 = _mm_clmulepi64_si128(_mm_and_si128(x, m32), pu, 0x10);
  __m128i t2 = _mm_clmulepi64_si128(_mm_and_si128(t1, m32), pu, 0x00);
  uint32_t c = (uint32_t)_mm_extract_epi32(_mm_xor_si128(x, t2), 1);
  return ~s8_update(c, p, n);
}
static int g_has_clmul = -1;
uint32_t tpzo_crc32_fast(const uint8_t* p, size_t n) {
  if (g_has_clmul < 0) {
    s8_init();
    __builtin_cpu_init();
    g_has_clmul = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1");
  }
  if (g_has_clmul && n >= 64) return clmul_crc(p, n);
  return ~s8_update(0xFFFFFFFFu, p, n);
}

/* One block's decoded view: Block{data, offsets} (src/block.rs:21-24). */
typedef struct {
  int status;
  uint32_t crc_actual, crc_expected;
  uint32_t n;
  const uint8_t* offs; /* n big-endian u16 */
  const uint8_t* data; /* entries region */
  size_t data_len;
} blockview;

/* compress::decode's codec step (src/block/compress.rs:95-113) for snappy (tag 2): the block's
 * Uncompress form (payload | crc | 1) in *buf (malloc'd, caller frees) and its length; the
 * block itself for any other tag. Returns 0, or TPZO_CODEC where snap returns Err. */
static int codec_step(const uint8_t* b, size_t len, uint8_t** buf, const uint8_t** out,
                      size_t* out_len) {
  *buf = NULL;
  *out = b;
  *out_len = len;
  if (len != 0 && b[len - 1] == 3) {
    /* lz4::block::decompress(data, None) (compress.rs:108-111): size prefix, then
     * LZ4_decompress_safe; the output is the decoded bytes (possibly fewer than the prefix) */
    int64_t size = 0;
    if (tpzo_lz4_prefixed_size(b, len - 1, &size) != 0) return TPZO_CODEC;
    const int64_t r = tpzo_lz4_decompress_safe(b + 4, (int64_t)len - 5, NULL, size);
    if (r < 0) return TPZO_CODEC;
    *buf = (uint8_t*)malloc((size_t)r + 1);
    tpzo_lz4_decompress_safe(b + 4, (int64_t)len - 5, *buf, size);
    (*buf)[r] = 1;
    *out = *buf;
    *out_len = (size_t)r + 1;
    return 0;
  }
  if (len == 0 || b[len - 1] != 2) return 0;
  uint64_t want = 0;
  if (tpzo_snappy_uncompressed_len(b, len - 1, &want) != 0) return TPZO_CODEC;
  *buf = (uint8_t*)malloc(want + 1);
  uint64_t got = 0;
  if (!*buf || tpzo_snappy_decompress(b, len - 1, *buf, want, &got) != 0) return TPZO_CODEC;
  (*buf)[got] = 1;
  *out = *buf;
  *out_len = got + 1;
  return 0;
}

/* compress::decode (src/block/compress.rs:95-113) + Block::decode (src/block.rs:46-65), on a
 * block whose codec step is done (tag 2 has become tag 1). */
static void block_decode(const uint8_t* b, size_t len, blockview* v) {
  memset(v, 0, sizeof(*v));
  if (len == 0) { v->status = TPZO_EMPTY; return; }             /* compress.rs:96-98 */
  uint8_t tag = b[len - 1];                                      /* compress.rs:99 */
  if (tag == 0 || tag > 3) { v->status = TPZO_BAD_TAG; return; } /* compress.rs:44-53,102 */
  if (tag != 1) { v->status = TPZO_UNSUPPORTED; return; }        /* lz4 */
  size_t dlen = len - 1;                                         /* compress.rs:100,103 */
  if (dlen < 4) { v->status = TPZO_MALFORMED; return; }          /* block.rs:49 split_to */
  size_t plen = dlen - 4;
  v->crc_expected = be32(b + plen);                              /* block.rs:51 */
  v->crc_actual = tpzo_crc32(b, plen);                           /* checksum.rs:13 */
  if (v->crc_actual != v->crc_expected) { v->status = TPZO_CHECKSUM; return; }
  if (plen < 2) { v->status = TPZO_MALFORMED; return; }          /* block.rs:54 get_u16 */
  v->n = be16(b);
  if (plen < 2 + 2 * (size_t)v->n) { v->status = TPZO_MALFORMED; return; } /* :56-59 */
  v->offs = b + 2;
  v->data = b + 2 + 2 * (size_t)v->n;                            /* block.rs:61-64 */
  v->data_len = plen - 2 - 2 * (size_t)v->n;
  v->status = TPZO_OK;
}

/* Entry i of a decoded block as BlockIterator reads it (src/block/iterator.rs:63-83 and the
 * bisection's key read, :95-98): `&data[offset..]` and get_u16 need offset + 2 <= L, `buf[..klen]`
 * needs offset + 2 + klen <= L (BAD_KEY otherwise), the second get_u16 and `buf[..vlen]` need
 * offset + 4 + klen + vlen <= L (BAD_VALUE otherwise). The readable parts are returned: key and
 * value for OK, the key for BAD_VALUE (with *vl = 0), nothing for BAD_KEY. */
static int entry_class(const blockview* v, uint32_t i, const uint8_t** k, uint32_t* kl,
                       const uint8_t** val, uint32_t* vl) {
  *kl = *vl = 0;
  *k = *val = v->data;
  size_t o = be16(v->offs + 2 * (size_t)i);                      /* :74 */
  if (o + 2 > v->data_len) return TPZO_ENTRY_BAD_KEY;            /* :75-77 */
  uint32_t klen = be16(v->data + o);
  if (o + 2 + klen > v->data_len) return TPZO_ENTRY_BAD_KEY;     /* :78 */
  *k = v->data + o + 2;
  *kl = klen;
  if (o + 2 + klen + 2 > v->data_len) return TPZO_ENTRY_BAD_VALUE; /* :80 */
  uint32_t vlen = be16(v->data + o + 2 + klen);
  if (o + 4 + klen + vlen > v->data_len) return TPZO_ENTRY_BAD_VALUE; /* :81-82 */
  *val = v->data + o + 4 + klen;
  *vl = vlen;
  return TPZO_ENTRY_OK;
}

/* BlockIterator::seek_to (src/block/iterator.rs:63-83) for index i < n; returns 0 when the
 * reference would panic (Buf::get_u16 underflow / slice out of range). */
static int entry_at(const blockview* v, uint32_t i, const uint8_t** k, uint32_t* kl,
                    const uint8_t** val, uint32_t* vl) {
  return entry_class(v, i, k, kl, val, vl) == TPZO_ENTRY_OK;
}

/* Decode a block and classify every entry the way an iteration over all indices would read it
 * (iterator.rs:63-83 reads entry i at offsets[i] with no ordering or disjointness check: entries
 * may overlap or repeat). Block::decode itself checks no entry (block.rs:46-65): a block with an
 * out-of-range entry is still Ok, reported TPZO_BAD_ENTRY here. kt / vt = the readable bytes. */
static void block_full(const uint8_t* b, size_t len, blockview* v, uint64_t* kt, uint64_t* vt) {
  block_decode(b, len, v);
  *kt = *vt = 0;
  if (v->status != TPZO_OK) return;
  for (uint32_t i = 0; i < v->n; i++) {
    const uint8_t *k, *val;
    uint32_t kl, vl;
    if (entry_class(v, i, &k, &kl, &val, &vl) != TPZO_ENTRY_OK) v->status = TPZO_BAD_ENTRY;
    *kt += kl;
    *vt += vl;
  }
}
static int block_ok(int st) { return st == TPZO_OK || st == TPZO_BAD_ENTRY; }

void tpzo_batch_sizes(const uint8_t* src, const uint64_t* ext, uint32_t n_blocks,
                      uint64_t* n_entries, uint64_t* key_bytes, uint64_t* val_bytes) {
  uint64_t ne = 0, kb = 0, vb = 0;
  for (uint32_t i = 0; i < n_blocks; i++) {
    blockview v;
    uint64_t kt = 0, vt = 0;
    uint8_t* buf;
    const uint8_t* blk;
    size_t blen;
    if (codec_step(src + ext[i], ext[i + 1] - ext[i], &buf, &blk, &blen) == 0) {
      block_full(blk, blen, &v, &kt, &vt);
      if (block_ok(v.status)) { ne += v.n; kb += kt; vb += vt; }
    }
    free(buf);
  }
  *n_entries = ne;
  *key_bytes = kb;
  *val_bytes = vb;
}

int tpzo_decode_batch(const uint8_t* src, const uint64_t* ext, uint32_t n_blocks,
                      uint8_t* status, uint32_t* crc_actual, uint32_t* crc_expected,
                      uint32_t* count, uint32_t* klen, uint32_t* vlen,
                      uint8_t* keys, uint8_t* vals, uint8_t* cls) {
  uint64_t e = 0, kp = 0, vp = 0;
  for (uint32_t i = 0; i < n_blocks; i++) {
    blockview v;
    uint64_t kt, vt;
    uint8_t* buf;
    const uint8_t* blk;
    size_t blen;
    const int cs = codec_step(src + ext[i], ext[i + 1] - ext[i], &buf, &blk, &blen);
    if (cs) {
      memset(&v, 0, sizeof v);
      v.status = cs;
    } else {
      block_full(blk, blen, &v, &kt, &vt);
    }
    status[i] = (uint8_t)v.status;
    crc_actual[i] = v.crc_actual;
    crc_expected[i] = v.crc_expected;
    count[i] = 0;
    if (!block_ok(v.status)) { free(buf); continue; }
    count[i] = v.n;
    for (uint32_t j = 0; j < v.n; j++, e++) {
      const uint8_t *k, *val;
      uint32_t kl, vl;
      const int c = entry_class(&v, j, &k, &kl, &val, &vl);
      if (cls) cls[e] = (uint8_t)c;
      klen[e] = kl;
      vlen[e] = vl;
      memcpy(keys + kp, k, kl);
      memcpy(vals + vp, val, vl);
      kp += kl;
      vp += vl;
    }
    free(buf);
  }
  return 0;
}

/* FileObject::open (file_object.rs:57-78): whole-file CRC, size excludes the trailer.
 * read_bloom (table.rs:75-87) and SsTable::open (table.rs:91-112): bloom_off, meta_off,
 * decode_block_meta (table.rs:49-59). */
int tpzo_sst_parse(const uint8_t* f, size_t len, uint64_t* ext, uint32_t ext_cap,
                   uint32_t* n_blocks, uint64_t* meta_off, uint64_t* bloom_off) {
  if (len < 4) return -2;
  size_t size = len - 4;
  if (tpzo_crc32(f, size) != be32(f + size)) return -1;
  if (size < 4) return -2;
  uint64_t bo = be32(f + size - 4);
  if (bo < 4 || bo + 4 > size) return -2;
  uint64_t mo = be32(f + bo - 4);
  if (mo > bo - 4) return -2;
  uint32_t nb = 0;
  size_t p = mo, end = bo - 4;
  while (p < end) {
    if (p + 6 > end) return -2;
    uint32_t off = be32(f + p);
    uint32_t kl = be16(f + p + 4);
    if (p + 6 + kl > end) return -2;
    if (nb >= ext_cap) return -3;
    ext[nb++] = off;
    p += 6 + kl;
  }
  if (nb >= ext_cap) return -3;
  ext[nb] = mo;
  *n_blocks = nb;
  *meta_off = mo;
  *bloom_off = bo;
  return 0;
}

/* ---- iterators ----------------------------------------------------------------------- */
struct tpzo_sst_iter {
  const uint8_t* file;
  uint64_t* ext;
  uint32_t nb;
  uint64_t* mk_off; /* first_key positions in the meta region */
  uint32_t* mk_len;
  /* SsTableIterator (table/iterator.rs:10-14) */
  uint32_t idx;
  /* BlockIterator (block/iterator.rs:9-14) over the current block */
  blockview blk;
  uint8_t* blkbuf; /* the current block's Uncompress form when it was snappy */
  uint32_t bidx;
  uint8_t *key, *val;
  size_t kl, vl, kcap, vcap;
};

static void set_bytes(uint8_t** dst, size_t* cap, size_t* len, const uint8_t* s, size_t n) {
  if (n > *cap) {
    *cap = n * 2 + 16;
    *dst = (uint8_t*)realloc(*dst, *cap);
  }
  if (n) memcpy(*dst, s, n);
  *len = n;
}

/* BlockIterator::seek_to (iterator.rs:63-83). Returns TPZO_PANIC where the reference panics
 * (an entry out of range: :74-82), else 0. */
static int biter_seek_to(tpzo_sst_iter* it, uint32_t i) {
  it->kl = it->vl = 0;
  if (i >= it->blk.n) { it->bidx = it->blk.n; return 0; }
  it->bidx = i;
  const uint8_t *k, *v;
  uint32_t kl, vl;
  if (!entry_at(&it->blk, i, &k, &kl, &v, &vl)) return TPZO_PANIC;
  set_bytes(&it->key, &it->kcap, &it->kl, k, kl);
  set_bytes(&it->val, &it->vcap, &it->vl, v, vl);
  return 0;
}

/* BlockIterator::seek_to_key (iterator.rs:91-109): lower-bound binary search; its key read
 * (:95-98) panics on a BAD_KEY entry, and the final seek_to on any bad entry. */
static int biter_seek_to_key(tpzo_sst_iter* it, const uint8_t* key, size_t klen) {
  uint32_t left = 0, right = it->blk.n;
  while (left < right) {
    uint32_t mid = (right - left) / 2 + left;
    const uint8_t *k, *v;
    uint32_t kl, vl;
    if (entry_class(&it->blk, mid, &k, &kl, &v, &vl) == TPZO_ENTRY_BAD_KEY) {
      it->bidx = mid;
      it->kl = it->vl = 0;
      return TPZO_PANIC;
    }
    size_t m = kl < klen ? kl : klen;
    int c = memcmp(k, key, m);
    if (c == 0) c = (kl > klen) - (kl < klen);
    if (c > 0) right = mid;
    else if (c < 0) left = mid + 1;
    else return biter_seek_to(it, mid);
  }
  return biter_seek_to(it, left);
}

/* SsTable::read_block (table.rs:154-164) into the iterator's current block. */
static int read_block(tpzo_sst_iter* it, uint32_t i) {
  free(it->blkbuf);
  const uint8_t* b;
  size_t len;
  if (codec_step(it->file + it->ext[i], it->ext[i + 1] - it->ext[i], &it->blkbuf, &b, &len)) {
    memset(&it->blk, 0, sizeof it->blk);
    it->blk.status = TPZO_CODEC;
    return -1;
  }
  block_decode(b, len, &it->blk);
  if (it->blk.status == TPZO_MALFORMED) return TPZO_PANIC;       /* block.rs:49-59 panics */
  return it->blk.status == TPZO_OK ? 0 : TPZO_ERR;
}

tpzo_sst_iter* tpzo_sst_iter_create(const uint8_t* file, size_t len) {
  uint32_t cap = (uint32_t)(len / 6 + 2), nb;
  uint64_t mo, bo;
  uint64_t* ext = (uint64_t*)malloc(sizeof(uint64_t) * cap);
  if (tpzo_sst_parse(file, len, ext, cap, &nb, &mo, &bo) != 0 || nb == 0) { free(ext); return NULL; }
  tpzo_sst_iter* it = (tpzo_sst_iter*)calloc(1, sizeof(*it));
  it->file = file;
  it->ext = ext;
  it->nb = nb;
  it->mk_off = (uint64_t*)malloc(sizeof(uint64_t) * nb);
  it->mk_len = (uint32_t*)malloc(sizeof(uint32_t) * nb);
  size_t p = mo;
  for (uint32_t i = 0; i < nb; i++) {
    it->mk_len[i] = be16(file + p + 4);
    it->mk_off[i] = p + 6;
    p += 6 + it->mk_len[i];
  }
  return it;
}

void tpzo_sst_iter_destroy(tpzo_sst_iter* it) {
  if (!it) return;
  free(it->ext);
  free(it->mk_off);
  free(it->mk_len);
  free(it->key);
  free(it->val);
  free(it->blkbuf);
  free(it);
}

/* seek_to_first_inner (table/iterator.rs:39-42) */
static int seek_first_inner(tpzo_sst_iter* it, uint32_t idx) {
  const int r = read_block(it, idx);
  if (r != 0) return r;
  return biter_seek_to(it, 0);
}

int tpzo_sst_iter_seek_to_first(tpzo_sst_iter* it) { /* table/iterator.rs:28-37 */
  it->idx = 0;
  return seek_first_inner(it, 0);
}

/* SsTable::find_block_idx (table.rs:178-182): partition_point(first_key <= key) - 1, sat. */
static uint32_t find_block_idx(const tpzo_sst_iter* it, const uint8_t* key, size_t klen) {
  uint32_t lo = 0, hi = it->nb;
  while (lo < hi) {
    uint32_t mid = lo + (hi - lo) / 2;
    const uint8_t* fk = it->file + it->mk_off[mid];
    size_t fl = it->mk_len[mid], m = fl < klen ? fl : klen;
    int c = memcmp(fk, key, m);
    if (c == 0) c = (fl > klen) - (fl < klen);
    if (c <= 0) lo = mid + 1; else hi = mid;
  }
  return lo ? lo - 1 : 0;
}

int tpzo_sst_iter_seek_to_key(tpzo_sst_iter* it, const uint8_t* key, size_t klen) {
  uint32_t idx = find_block_idx(it, key, klen);                   /* :55 */
  it->idx = idx;
  int r = read_block(it, idx);                                    /* :56 */
  if (r != 0) return r;
  r = biter_seek_to_key(it, key, klen);                           /* :57 */
  if (r != 0) return r;
  if (it->kl == 0 && idx + 1 < it->nb) {                          /* :58-61 */
    idx += 1;
    it->idx = idx;
    r = seek_first_inner(it, idx);
    if (r != 0) return r;
  }
  return 0;
}

int tpzo_sst_iter_next(tpzo_sst_iter* it) { /* table/iterator.rs:88-95 */
  const int r = biter_seek_to(it, it->bidx + 1);
  if (r != 0) return r;
  if (it->kl == 0 && it->idx < it->nb - 1) {
    it->idx += 1;
    return seek_first_inner(it, it->idx);
  }
  return 0;
}

/* SsTable::init_samllest_biggest_key (src/table.rs:143-151). */
int tpzo_sst_biggest_key(tpzo_sst_iter* it, const uint8_t** key, size_t* len) {
  *key = NULL;
  *len = 0;
  int r = read_block(it, it->nb - 1);                             /* :145 */
  if (r != 0) return r;
  r = biter_seek_to(it, 0);                                       /* :146 */
  if (r != 0) return r;
  if (it->blk.n == 0) return TPZO_PANIC;                          /* :147, iterator.rs:60 */
  r = biter_seek_to(it, it->blk.n - 1);
  if (r != 0) return r;
  if (it->kl == 0) return TPZO_PANIC;                             /* :148 assert!(is_valid) */
  *key = it->key;
  *len = it->kl;
  return 0;
}

int tpzo_sst_iter_is_valid(const tpzo_sst_iter* it) { return it->kl != 0; }
const uint8_t* tpzo_sst_iter_key(const tpzo_sst_iter* it, size_t* len) { *len = it->kl; return it->key; }
const uint8_t* tpzo_sst_iter_value(const tpzo_sst_iter* it, size_t* len) { *len = it->vl; return it->val; }
uint32_t tpzo_sst_iter_block_idx(const tpzo_sst_iter* it) { return it->idx; }

/* ---- CPU baseline ------------------------------------------------------------------------ */
typedef struct {
  int fd;
  uint64_t* ext;
  uint32_t nb;
} sstfile;

/* FileObject::open + SsTable::open on a path: whole-file read and CRC (file_object.rs:57-78). */
static int sst_file_open(const char* path, sstfile* s) {
  int fd = open(path, O_RDONLY);
  if (fd < 0) return -1;
  off_t len = lseek(fd, 0, SEEK_END);
  uint8_t* buf = (uint8_t*)malloc((size_t)len);
  if (pread(fd, buf, (size_t)len, 0) != len) { free(buf); close(fd); return -1; }
  uint32_t cap = (uint32_t)(len / 6 + 2);
  s->ext = (uint64_t*)malloc(sizeof(uint64_t) * cap);
  uint64_t mo, bo;
  int rc = tpzo_sst_parse(buf, (size_t)len, s->ext, cap, &s->nb, &mo, &bo);
  free(buf);
  if (rc) { close(fd); free(s->ext); return -1; }
  s->fd = fd;
  return 0;
}

/* One `create_and_read` pass (benches/sstable_iter_read.rs:70-76): for every block a fresh
 * Vec + pread (file_object.rs:23-27), the codec's BytesMut copy (compress.rs:103), CRC
 * (block.rs:52), offsets Vec (block.rs:56-59); per entry key/value to_vec (iterator.rs:78,82).
 * The per-block and per-entry allocations are kept: they are what the reference spends. */
static uint64_t iter_read_pass(const sstfile* s, volatile uint64_t* sink, uint64_t* bytes) {
  uint64_t ents = 0, by = 0, acc = 0;
  for (uint32_t b = 0; b < s->nb; b++) {
    size_t len = s->ext[b + 1] - s->ext[b];
    uint8_t* raw = (uint8_t*)malloc(len ? len : 1);
    if (pread(s->fd, raw, len, (off_t)s->ext[b]) != (ssize_t)len) { free(raw); return ents; }
    by += len;
    if (len == 0) { free(raw); continue; }
    /* compress::decode (compress.rs:95-113): the codec's output buffer (one decode pass, as
     * snap / LZ4_decompress_safe do), or the BytesMut copy of an Uncompress payload */
    const uint8_t tag = raw[len - 1];
    uint8_t* data = NULL;
    size_t dlen = 0;
    if (tag == 1) {
      dlen = len - 1;
      data = (uint8_t*)malloc(dlen ? dlen : 1);
      memcpy(data, raw, dlen);
    } else if (tag == 2) {
      uint64_t want = 0, got = 0;
      if (tpzo_snappy_uncompressed_len(raw, len - 1, &want) == 0) {
        data = (uint8_t*)malloc(want ? want : 1);
        if (tpzo_snappy_decompress(raw, len - 1, data, want, &got) != 0) { free(data); data = NULL; }
        dlen = got;
      }
    } else if (tag == 3) {
      int64_t size = 0;
      if (tpzo_lz4_prefixed_size(raw, len - 1, &size) == 0) {
        data = (uint8_t*)malloc(size ? (size_t)size : 1);
        const int64_t r = tpzo_lz4_decompress_safe(raw + 4, (int64_t)len - 5, data, size);
        if (r < 0) { free(data); data = NULL; }
        dlen = r < 0 ? 0 : (size_t)r;
      }
    }
    free(raw);
    if (!data) continue;
    if (dlen < 4) { free(data); continue; }
    size_t plen = dlen - 4;
    if (tpzo_crc32_fast(data, plen) != be32(data + plen) || plen < 2) { free(data); continue; }
    uint32_t n = be16(data);
    if (plen < 2 + 2 * (size_t)n) { free(data); continue; }
    uint16_t* offs = (uint16_t*)malloc(sizeof(uint16_t) * (n ? n : 1));
    for (uint32_t i = 0; i < n; i++) offs[i] = (uint16_t)be16(data + 2 + 2 * i);
    const uint8_t* d = data + 2 + 2 * (size_t)n;
    size_t dl = plen - 2 - 2 * (size_t)n;
    for (uint32_t i = 0; i < n; i++) {
      size_t o = offs[i];
      if (o + 2 > dl) break;
      uint32_t kl = be16(d + o);
      if (o + 4 + kl > dl) break;
      uint32_t vl = be16(d + o + 2 + kl);
      if (o + 4 + kl + vl > dl) break;
      if (kl == 0) break; /* is_valid == key non-empty (iterator.rs:50-52) */
      uint8_t* k = (uint8_t*)malloc(kl);
      memcpy(k, d + o + 2, kl);
      uint8_t* v = (uint8_t*)malloc(vl ? vl : 1);
      memcpy(v, d + o + 4 + kl, vl);
      acc += k[0] + (vl ? v[vl - 1] : 0);
      free(k);
      free(v);
      ents++;
    }
    free(offs);
    free(data);
  }
  *sink += acc;
  *bytes = by;
  return ents;
}

typedef struct {
  const sstfile* files;
  uint32_t first, step, n, iters;
  uint64_t bytes, entries;
} worker;

static volatile uint64_t g_sink;

static void* worker_main(void* arg) {
  worker* w = (worker*)arg;
  for (uint32_t it = 0; it < w->iters; it++)
    for (uint32_t f = w->first; f < w->n; f += w->step) {
      uint64_t by = 0;
      uint64_t e = iter_read_pass(&w->files[f], &g_sink, &by);
      if (it == 0) { w->bytes += by; w->entries += e; }
    }
  return NULL;
}

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

double tpzo_bench_iter_read(const char* const* paths, uint32_t n_paths, uint32_t threads,
                            uint32_t iters, uint64_t* bytes, uint64_t* entries) {
  sstfile* files = (sstfile*)calloc(n_paths, sizeof(sstfile));
  for (uint32_t i = 0; i < n_paths; i++)
    if (sst_file_open(paths[i], &files[i]) != 0) { free(files); return -1.0; }
  if (threads == 0) threads = 1;
  worker* ws = (worker*)calloc(threads, sizeof(worker));
  pthread_t* th = (pthread_t*)calloc(threads, sizeof(pthread_t));
  double t0 = now_s();
  for (uint32_t t = 0; t < threads; t++) {
    ws[t] = (worker){files, t, threads, n_paths, iters, 0, 0};
    pthread_create(&th[t], NULL, worker_main, &ws[t]);
  }
  uint64_t by = 0, en = 0;
  for (uint32_t t = 0; t < threads; t++) {
    pthread_join(th[t], NULL);
    by += ws[t].bytes;
    en += ws[t].entries;
  }
  double dt = now_s() - t0;
  for (uint32_t i = 0; i < n_paths; i++) { close(files[i].fd); free(files[i].ext); }
  free(files);
  free(ws);
  free(th);
  *bytes = by;
  *entries = en;
  return dt;
}

/* ---- write side: SsTableBuilder's data region with CompressOptions::Uncompress ------------
 * The checker for tpz_plan_blocks / tpz_encode_blocks. Restates, entry by entry:
 *   BlockBuilder::add           src/block/builder.rs:26-41 (assert key non-empty; full when
 *                               encode_len + size + 2 > target_size; offsets as u16)
 *   SsTableBuilder::add         src/table/builder.rs:49-64 (a full block is built, then the
 *                               entry is added again: an entry that fits no block recurses
 *                               forever in the reference -> -2 here)
 *   SsTableBuilder::block_build src/table/builder.rs:66-85 (BlockMeta::offset = data.len())
 *   Block::encode               src/block.rs:31-44 (n u16 BE, offsets u16 BE, data, crc BE)
 *   Entry::encode               src/block/builder.rs:72-81 (klen u16 BE, key, vlen u16 BE, value)
 *   compress::encode Uncompress src/block/compress.rs:85-89 (tag byte 1)
 * Returns the number of blocks, -1 when out_cap / ext_cap are too small, -2 with *bad = the
 * entry index for an empty key or an entry no block holds. ext gets n_blocks + 1 offsets,
 * first the first entry of every block. */
typedef struct {
  uint32_t target, size;       /* BlockBuilder { target_size, size } */
  uint64_t first, count;       /* entries [first, first + count) (data + offsets) */
} tpzo_bb;

static int bb_add(tpzo_bb* b, uint64_t klen, uint64_t vlen) {
  const uint64_t enc = 2 + klen + 2 + vlen;           /* Entry::encode_len */
  if (enc + b->size + 2 > b->target) return 0;
  b->size += (uint32_t)enc;
  b->count++;
  return 1;
}

static void put_be16(uint8_t* p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }

int64_t tpzo_build_blocks(const uint8_t* keys, const uint64_t* kpos, const uint8_t* vals,
                          const uint64_t* vpos, uint64_t n, uint32_t block_size, uint8_t* out,
                          uint64_t out_cap, uint64_t* ext, uint64_t* first, uint64_t ext_cap,
                          uint64_t* bad) {
  uint64_t len = 0, nb = 0, e = 0;
  tpzo_bb b = {block_size, 0, 0, 0};
  for (;;) {
    const int more = e < n;
    if (more) {
      const uint64_t kl = kpos[e + 1] - kpos[e], vl = vpos[e + 1] - vpos[e];
      if (kl == 0) { *bad = e; return -2; }
      if (bb_add(&b, kl, vl)) { e++; continue; }
      if (b.count == 0) { *bad = e; return -2; }
    }
    if (b.count) {                                      /* block_build */
      const uint64_t blen = 2 + 2 * b.count + b.size + 5;
      if (len + blen > out_cap || nb + 2 > ext_cap) return -1;
      uint8_t* p = out + len;
      put_be16(p, (uint32_t)b.count);
      uint32_t off = 0;
      uint8_t* d = p + 2 + 2 * b.count;
      for (uint64_t i = 0; i < b.count; i++) {
        const uint64_t x = b.first + i, kl = kpos[x + 1] - kpos[x], vl = vpos[x + 1] - vpos[x];
        put_be16(p + 2 + 2 * i, off);
        put_be16(d + off, (uint32_t)kl);
        memcpy(d + off + 2, keys + kpos[x], kl);
        put_be16(d + off + 2 + kl, (uint32_t)vl);
        memcpy(d + off + 4 + kl, vals + vpos[x], vl);
        off += (uint32_t)(4 + kl + vl);
      }
      const uint64_t plen = 2 + 2 * b.count + b.size;
      const uint32_t crc = tpzo_crc32(p, plen);
      p[plen] = (uint8_t)(crc >> 24); p[plen + 1] = (uint8_t)(crc >> 16);
      p[plen + 2] = (uint8_t)(crc >> 8); p[plen + 3] = (uint8_t)crc;
      p[plen + 4] = 1;
      ext[nb] = len;
      first[nb] = b.first;
      nb++;
      len += blen;
    }
    if (!more) break;
    b.size = 0; b.first = e; b.count = 0;
  }
  ext[nb] = len;
  first[nb] = n;
  return (int64_t)nb;
}
