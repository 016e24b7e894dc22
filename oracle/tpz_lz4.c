/*
 * tpz_lz4.c — CPU restatement of the LZ4 block format as topazdb's block codec 3 uses it.
 * TEST INFRASTRUCTURE ONLY (see tpz_oracle.h): the checker for the device decompressor, never
 * the product.
 *
 * The reference calls the `lz4` crate ("*" in Cargo.toml:18, unpinned), which binds liblz4:
 *   encode: lz4::block::compress(data, None, true)   src/block/compress.rs:73-77
 *           (prepend_size: 4-byte little-endian uncompressed size, then LZ4_compress_default)
 *   decode: lz4::block::decompress(data, None)?      src/block/compress.rs:108-111
 *           size = the i32 LE prefix (Err if the source is shorter than 4 bytes, if size < 0,
 *           or if LZ4_compressBound(size) <= 0, i.e. size > 0x7E000000); then
 *           LZ4_decompress_safe(src + 4, dst, len - 4, size): Err if it returns < 0, else the
 *           output is its first `ret` bytes (ret may be below size).
 * The decoder's acceptance rules are liblz4's, restated here from LZ4_decompress_generic as
 * liblz4 1.9.3 (the version in this image, /usr/lib/x86_64-linux-gnu/liblz4.so.1.9.3) builds it
 * for LZ4_decompress_safe: the fast loop while >= 64 output bytes remain (FASTLOOP_SAFE_DISTANCE),
 * then the safe loop with its two-stage shortcut; the two loops accept slightly different inputs
 * near the ends of the buffers, so both are restated. tests/test_lz4_oracle.py pins this
 * restatement against liblz4 itself (valid streams, corruptions, crafted edge streams).
 *
 * Format: sequences of token (literal length << 4 | match length - 4), literal-length extension
 * bytes (while 255), literals, a 2-byte LE offset, match-length extension bytes; the last
 * sequence is literals only. A match repeats the bytes `offset` back (overlap = periodic);
 * liblz4 1.9.3 fills an offset-0 match with zeros.
 */
#include <stdint.h>
#include <string.h>

#include "tpz_oracle.h"

enum { MINMATCH = 4, LASTLITERALS = 5, MFLIMIT = 12, FASTLOOP = 64, RUN_MASK = 15, ML_MASK = 15 };

/* A match of `len` bytes at out[op] from `off` bytes back (off <= op checked by the caller). */
static void match_copy(uint8_t* out, int64_t op, int64_t off, int64_t len) {
  if (!out) return;
  if (off == 0) {
    memset(out + op, 0, (size_t)len);
    return;
  }
  for (int64_t k = 0; k < len; k++) out[op + k] = out[op + k - off];
}

static void lit_copy(uint8_t* out, int64_t op, const uint8_t* in, int64_t ip, int64_t len) {
  if (out) memcpy(out + op, in + ip, (size_t)len);
}

int64_t tpzo_lz4_decompress_safe(const uint8_t* in, int64_t src_size, uint8_t* out,
                                 int64_t out_size) {
  if (out_size == 0) return (src_size == 1 && in[0] == 0) ? 0 : -1;
  if (src_size == 0) return -1;
  const int64_t iend = src_size, oend = out_size;
  const int64_t shortiend = iend - 14 - 2, shortoend = oend - 14 - 18;
  int64_t ip = 0, op = 0, lit = 0, ml = 0, off = 0, match = 0, cpy = 0;
  uint32_t token = 0;

  if (oend - op >= FASTLOOP) {
    /* fast loop: while FASTLOOP_SAFE_DISTANCE output bytes remain */
    for (;;) {
      token = in[ip++];
      lit = token >> 4;
      if (lit == RUN_MASK) {
        if (ip >= iend - RUN_MASK) return -1;                 /* initial_error */
        uint32_t s;
        do {
          s = in[ip++];
          lit += s;
          if (ip >= iend - RUN_MASK) break;                   /* loop_error: not fatal here */
        } while (s == 255);
        cpy = op + lit;
        if (cpy > oend - 32 || ip + lit > iend - 32) goto safe_literal_copy;
        lit_copy(out, op, in, ip, lit);
        ip += lit;
        op = cpy;
      } else {
        cpy = op + lit;
        if (ip > iend - 17) goto safe_literal_copy;
        lit_copy(out, op, in, ip, lit);
        ip += lit;
        op = cpy;
      }
      off = (int64_t)in[ip] | (int64_t)in[ip + 1] << 8;
      ip += 2;
      match = op - off;
      ml = token & ML_MASK;
      if (ml == ML_MASK) {
        if (match < 0) return -1;
        uint32_t s;
        do {
          s = in[ip++];
          ml += s;
          if (ip >= iend - LASTLITERALS + 1) return -1;
        } while (s == 255);
        ml += MINMATCH;
        if (op + ml >= oend - FASTLOOP) goto safe_match_copy;
      } else {
        ml += MINMATCH;
        if (op + ml >= oend - FASTLOOP) goto safe_match_copy;
        if (match >= 0 && off >= 8) {
          match_copy(out, op, off, ml);
          op += ml;
          continue;
        }
      }
      if (match < 0) return -1;
      match_copy(out, op, off, ml);
      op += ml;
    }
  }

  /* safe loop */
  for (;;) {
    token = in[ip++];
    lit = token >> 4;
    if (lit != RUN_MASK && ip < shortiend && op <= shortoend) {
      /* two-stage shortcut: no end-of-buffer checks on this sequence's literals */
      lit_copy(out, op, in, ip, lit);
      op += lit;
      ip += lit;
      ml = token & ML_MASK;
      off = (int64_t)in[ip] | (int64_t)in[ip + 1] << 8;
      ip += 2;
      match = op - off;
      if (ml != ML_MASK && off >= 8 && match >= 0) {
        match_copy(out, op, off, ml + MINMATCH);
        op += ml + MINMATCH;
        continue;
      }
      goto copy_match;
    }
    if (lit == RUN_MASK) {
      if (ip >= iend - RUN_MASK) return -1;
      uint32_t s;
      do {
        s = in[ip++];
        lit += s;
        if (ip >= iend - RUN_MASK) break;
      } while (s == 255);
    }
    cpy = op + lit;
  safe_literal_copy:
    if (cpy > oend - MFLIMIT || ip + lit > iend - (2 + 1 + LASTLITERALS)) {
      /* must be the last sequence: it consumes the input exactly and fits the output */
      if (ip + lit != iend || cpy > oend) return -1;
      lit_copy(out, op, in, ip, lit);
      ip += lit;
      op += lit;
      break;
    }
    lit_copy(out, op, in, ip, lit);
    ip += lit;
    op = cpy;
    off = (int64_t)in[ip] | (int64_t)in[ip + 1] << 8;
    ip += 2;
    match = op - off;
    ml = token & ML_MASK;
  copy_match:
    if (ml == ML_MASK) {
      uint32_t s;
      do {
        s = in[ip++];
        ml += s;
        if (ip >= iend - LASTLITERALS + 1) return -1;
      } while (s == 255);
    }
    ml += MINMATCH;
  safe_match_copy:
    if (match < 0) return -1;
    cpy = op + ml;
    if (cpy > oend - LASTLITERALS) return -1;   /* the last 5 bytes must be literals */
    match_copy(out, op, off, ml);
    op = cpy;
  }
  return op;
}

int tpzo_lz4_prefixed_size(const uint8_t* src, size_t n, int64_t* size) {
  if (n < 4) return -1;                                  /* "must at least contain size prefix" */
  const int32_t s = (int32_t)((uint32_t)src[0] | (uint32_t)src[1] << 8 | (uint32_t)src[2] << 16 |
                              (uint32_t)src[3] << 24);
  if (s < 0 || s > 0x7E000000) return -1;                /* negative / LZ4_compressBound <= 0 */
  *size = s;
  return 0;
}

/* Greedy LZ4 block compressor over a 4-byte hash (for fixtures and benches), keeping the
 * format's end rules: the last match starts at least MFLIMIT (12) bytes before the end and
 * the last 5 bytes are literals. `mode` 1 disables matches (literals only). */
size_t tpzo_lz4_compress(const uint8_t* src, size_t n, uint8_t* dst, int mode) {
  enum { HBITS = 14 };
  static uint32_t table[1 << HBITS];
  memset(table, 0xFF, sizeof(table));
  size_t p = 0, anchor = 0, i = 0;
  const size_t mflimit = n > MFLIMIT ? n - MFLIMIT : 0;
  const size_t matchlimit = n > LASTLITERALS ? n - LASTLITERALS : 0;
  while (mode != 1 && i + 4 <= n && i < mflimit) {
    uint32_t w;
    memcpy(&w, src + i, 4);
    const uint32_t h = (w * 2654435761u) >> (32 - HBITS);
    const uint32_t cand = table[h];
    table[h] = (uint32_t)i;
    uint32_t cw = 0;
    if (cand != 0xFFFFFFFFu) memcpy(&cw, src + cand, 4);
    if (cand == 0xFFFFFFFFu || cw != w || i - cand > 65535) {
      i++;
      continue;
    }
    size_t m = 4;
    while (i + m < matchlimit && src[cand + m] == src[i + m]) m++;
    /* sequence: literals [anchor, i), match (i - cand, m) */
    const size_t ll = i - anchor, mlc = m - MINMATCH;
    uint8_t* tok = dst + p++;
    *tok = (uint8_t)((ll >= RUN_MASK ? RUN_MASK : ll) << 4 | (mlc >= ML_MASK ? ML_MASK : mlc));
    if (ll >= RUN_MASK) {
      size_t r = ll - RUN_MASK;
      for (; r >= 255; r -= 255) dst[p++] = 255;
      dst[p++] = (uint8_t)r;
    }
    memcpy(dst + p, src + anchor, ll);
    p += ll;
    const size_t o = i - cand;
    dst[p++] = (uint8_t)o;
    dst[p++] = (uint8_t)(o >> 8);
    if (mlc >= ML_MASK) {
      size_t r = mlc - ML_MASK;
      for (; r >= 255; r -= 255) dst[p++] = 255;
      dst[p++] = (uint8_t)r;
    }
    i += m;
    anchor = i;
  }
  /* last literals */
  const size_t ll = n - anchor;
  dst[p++] = (uint8_t)((ll >= RUN_MASK ? RUN_MASK : ll) << 4);
  if (ll >= RUN_MASK) {
    size_t r = ll - RUN_MASK;
    for (; r >= 255; r -= 255) dst[p++] = 255;
    dst[p++] = (uint8_t)r;
  }
  memcpy(dst + p, src + anchor, ll);
  return p + ll;
}
