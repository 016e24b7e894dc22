/*
 * tpz_snappy.c — CPU restatement of the snappy raw format used by topazdb's block codec 2.
 * TEST INFRASTRUCTURE ONLY (see tpz_oracle.h): the checker for the device decompressor, never
 * the product.
 *
 * The reference calls the `snap` crate ("*" in Cargo.toml:17, unpinned):
 *   encode: snap::raw::Encoder::new().compress_vec(data)      src/block/compress.rs:66-71
 *   decode: snap::raw::Decoder::new().decompress_vec(data)?   src/block/compress.rs:104-107
 * No snappy implementation exists in this image, so this file restates the published raw
 * format (google/snappy format_description.txt) and snap's decoder checks:
 *   stream   = varint(uncompressed length) element*
 *   element  = tag byte, tag & 3:
 *     0 literal : len-1 = tag >> 2 when < 60; else (tag >> 2) - 59 = 1..4 little-endian bytes
 *                 follow holding len-1; then len literal bytes
 *     1 copy    : len = 4 + ((tag >> 2) & 7), offset = (tag >> 5) << 8 | next byte
 *     2 copy    : len = 1 + (tag >> 2), offset = next 2 bytes little-endian
 *     3 copy    : len = 1 + (tag >> 2), offset = next 4 bytes little-endian
 *   a copy repeats the `len` bytes starting `offset` bytes back (they may overlap the output).
 * snap rejects (Err): a truncated or over-long varint; a declared length above 2^32 - 1; a
 * literal or copy running past the input or past the declared length; offset 0 or an offset
 * beyond the bytes produced; an output shorter than declared.
 */
#include <stdint.h>
#include <string.h>

#include "tpz_oracle.h"

/* The varint preamble. Returns the header length, 0 on error. */
static size_t snappy_header(const uint8_t* s, size_t n, uint64_t* len) {
  uint64_t v = 0;
  for (size_t i = 0; i < n && i < 10; i++) {
    v |= (uint64_t)(s[i] & 0x7F) << (7 * i);
    if (!(s[i] & 0x80)) {
      if (v > 0xFFFFFFFFull) return 0;
      *len = v;
      return i + 1;
    }
  }
  return 0;
}

int tpzo_snappy_uncompressed_len(const uint8_t* src, size_t n, uint64_t* len) {
  return snappy_header(src, n, len) ? 0 : -1;
}

int tpzo_snappy_decompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap,
                           uint64_t* out_len) {
  uint64_t want;
  size_t ip = snappy_header(src, n, &want);
  if (!ip || want > cap) return -1;
  uint64_t d = 0;
  while (ip < n) {
    const uint32_t tag = src[ip++];
    uint64_t len, off;
    switch (tag & 3) {
      case 0: {
        len = (tag >> 2) + 1;
        if ((tag >> 2) >= 60) {
          const size_t nb = (tag >> 2) - 59;
          if (ip + nb > n) return -1;
          uint64_t v = 0;
          for (size_t k = 0; k < nb; k++) v |= (uint64_t)src[ip + k] << (8 * k);
          ip += nb;
          len = v + 1;
        }
        if (ip + len > n || d + len > want) return -1;
        memcpy(dst + d, src + ip, len);
        ip += len;
        d += len;
        continue;
      }
      case 1:
        if (ip + 1 > n) return -1;
        len = 4 + ((tag >> 2) & 7);
        off = ((uint64_t)(tag >> 5) << 8) | src[ip];
        ip += 1;
        break;
      case 2:
        if (ip + 2 > n) return -1;
        len = 1 + (tag >> 2);
        off = (uint64_t)src[ip] | (uint64_t)src[ip + 1] << 8;
        ip += 2;
        break;
      default:
        if (ip + 4 > n) return -1;
        len = 1 + (tag >> 2);
        off = (uint64_t)src[ip] | (uint64_t)src[ip + 1] << 8 | (uint64_t)src[ip + 2] << 16 |
              (uint64_t)src[ip + 3] << 24;
        ip += 4;
        break;
    }
    if (off == 0 || off > d || d + len > want) return -1;
    for (uint64_t k = 0; k < len; k++) dst[d + k] = dst[d - off + k];  /* byte order: overlaps */
    d += len;
  }
  if (d != want) return -1;
  *out_len = d;
  return 0;
}

/* ---- a compressor for fixtures (any valid stream decodes identically) ---------------------
 * Greedy LZ77 over a 4-byte hash, as the snappy format intends; `mode` varies the element mix so
 * fixtures exercise every element kind: 0 = copy-1 when it fits else copy-2, 1 = copy-2 only,
 * 2 = copy-4 only, 3 = literals only (long literals use 1-4 length bytes). */
static size_t put_literal(uint8_t* o, const uint8_t* s, size_t len) {
  size_t p = 0;
  const size_t v = len - 1;
  if (v < 60) {
    o[p++] = (uint8_t)(v << 2);
  } else {
    int nb = v < (1u << 8) ? 1 : v < (1u << 16) ? 2 : v < (1u << 24) ? 3 : 4;
    o[p++] = (uint8_t)((59 + nb) << 2);
    for (int k = 0; k < nb; k++) o[p++] = (uint8_t)(v >> (8 * k));
  }
  memcpy(o + p, s, len);
  return p + len;
}

static size_t put_copy(uint8_t* o, uint64_t off, size_t len, int mode) {
  size_t p = 0;
  while (len > 0) {
    size_t l = len > 64 ? 64 : len;
    if (len > 64 && len - 64 < 4) l = 60;  /* keep the remainder >= 4 for copy-1 */
    if (mode == 0 && l >= 4 && l <= 11 && off < 2048) {
      o[p++] = (uint8_t)(1 | ((l - 4) << 2) | ((off >> 8) << 5));
      o[p++] = (uint8_t)off;
    } else if (mode != 2 && off < 65536) {
      o[p++] = (uint8_t)(2 | ((l - 1) << 2));
      o[p++] = (uint8_t)off;
      o[p++] = (uint8_t)(off >> 8);
    } else {
      o[p++] = (uint8_t)(3 | ((l - 1) << 2));
      for (int k = 0; k < 4; k++) o[p++] = (uint8_t)(off >> (8 * k));
    }
    len -= l;
  }
  return p;
}

size_t tpzo_snappy_compress(const uint8_t* src, size_t n, uint8_t* dst, int mode) {
  size_t p = 0;
  uint64_t v = n;
  do {
    dst[p++] = (uint8_t)((v & 0x7F) | (v > 0x7F ? 0x80 : 0));
    v >>= 7;
  } while (v);
  enum { HBITS = 14 };
  static __thread uint32_t table[1 << HBITS];
  memset(table, 0xFF, sizeof table);
  size_t lit = 0, i = 0;
  while (mode != 3 && i + 4 <= n) {
    uint32_t w;
    memcpy(&w, src + i, 4);
    const uint32_t h = (w * 0x1E35A7BDu) >> (32 - HBITS);
    const uint32_t cand = table[h];
    table[h] = (uint32_t)i;
    uint32_t cw = 0;
    if (cand != 0xFFFFFFFFu) memcpy(&cw, src + cand, 4);
    if (cand == 0xFFFFFFFFu || cw != w || (mode != 2 && i - cand >= 65536)) {
      i++;
      continue;
    }
    size_t m = 4;
    while (i + m < n && src[cand + m] == src[i + m]) m++;
    if (i > lit) p += put_literal(dst + p, src + lit, i - lit);
    p += put_copy(dst + p, i - cand, m, mode);
    i += m;
    lit = i;
  }
  if (n > lit) p += put_literal(dst + p, src + lit, n - lit);
  return p;
}
