// tpz_host_builder.cpp — host write side: BlockBuilder + SsTableBuilder block packing.
//
// Restates src/block/builder.rs:26-85 (fill rule, Entry::encode), src/block.rs:31-44
// (Block::encode: u16 n | u16 off[n] | entries | u32 crc32 | codec tag) and
// src/table/builder.rs:49-85 (SsTableBuilder::add / block_build: one block after another,
// back to back) for the Uncompress codec (src/block/compress.rs:85-89), and re-encodes blocks
// with the Snappy codec (compress.rs:66-71; a greedy LZ77 emitter of the snappy raw format, the
// role snap::raw::Encoder plays). It produces SST data regions for bench.py and for the table
// facade; it is not on the decode path.
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/tpz_gpu.h"

namespace {

struct Crc32 {
  uint32_t t[8][256];
  Crc32() {
    for (uint32_t b = 0; b < 256; b++) {
      uint32_t c = b;
      for (int i = 0; i < 8; i++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
      t[0][b] = c;
    }
    for (int k = 1; k < 8; k++)
      for (uint32_t b = 0; b < 256; b++) t[k][b] = (t[k - 1][b] >> 8) ^ t[0][t[k - 1][b] & 0xFF];
  }
  // crc32fast-compatible CRC-32/ISO-HDLC, slicing-by-8 (src/checksum.rs:6-10)
  uint32_t operator()(const uint8_t* p, size_t n) const {
    uint32_t c = 0xFFFFFFFFu;
    while (n >= 8) {
      uint32_t lo, hi;
      std::memcpy(&lo, p, 4);
      std::memcpy(&hi, p + 4, 4);
      lo ^= c;
      c = t[7][lo & 0xFF] ^ t[6][(lo >> 8) & 0xFF] ^ t[5][(lo >> 16) & 0xFF] ^ t[4][lo >> 24] ^
          t[3][hi & 0xFF] ^ t[2][(hi >> 8) & 0xFF] ^ t[1][(hi >> 16) & 0xFF] ^ t[0][hi >> 24];
      p += 8;
      n -= 8;
    }
    while (n--) c = (c >> 8) ^ t[0][(c ^ *p++) & 0xFF];
    return ~c;
  }
};

const Crc32& crc() {
  static const Crc32 c;
  return c;
}

inline void put16(uint8_t* p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
inline void put32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}

// Snappy raw-format encoder: varint length, then literals and copies found with a 4-byte hash
// (copy-1 for lengths 4..11 within 2 KiB, else copy-2; offsets < 64 KiB). Returns the length.
size_t snappy_encode(const uint8_t* s, size_t n, uint8_t* o) {
  size_t p = 0;
  for (uint64_t v = n;; v >>= 7) {
    o[p++] = (uint8_t)((v & 0x7F) | (v > 0x7F ? 0x80 : 0));
    if (v <= 0x7F) break;
  }
  auto literal = [&](size_t lo, size_t hi) {
    if (hi <= lo) return;
    const size_t v = hi - lo - 1;
    if (v < 60) {
      o[p++] = (uint8_t)(v << 2);
    } else {
      const int nb = v < (1u << 8) ? 1 : v < (1u << 16) ? 2 : v < (1u << 24) ? 3 : 4;
      o[p++] = (uint8_t)((59 + nb) << 2);
      for (int k = 0; k < nb; k++) o[p++] = (uint8_t)(v >> (8 * k));
    }
    std::memcpy(o + p, s + lo, hi - lo);
    p += hi - lo;
  };
  constexpr int kBits = 13;
  thread_local std::vector<int32_t> table(1 << kBits);
  std::fill(table.begin(), table.end(), -1);
  size_t lit = 0, i = 0;
  while (i + 4 <= n) {
    uint32_t w;
    std::memcpy(&w, s + i, 4);
    const uint32_t h = (w * 0x1E35A7BDu) >> (32 - kBits);
    const int32_t c = table[h];
    table[h] = (int32_t)i;
    uint32_t cw;
    if (c < 0 || i - (size_t)c >= 65536 || (std::memcpy(&cw, s + c, 4), cw != w)) {
      i++;
      continue;
    }
    size_t m = 4;
    while (i + m < n && s[c + m] == s[i + m]) m++;
    literal(lit, i);
    const size_t off = i - (size_t)c;
    for (size_t rem = m; rem;) {
      size_t l = rem > 64 ? (rem - 64 < 4 ? 60 : 64) : rem;
      if (l >= 4 && l <= 11 && off < 2048) {
        o[p++] = (uint8_t)(1 | ((l - 4) << 2) | ((off >> 8) << 5));
        o[p++] = (uint8_t)off;
      } else {
        o[p++] = (uint8_t)(2 | ((l - 1) << 2));
        o[p++] = (uint8_t)off;
        o[p++] = (uint8_t)(off >> 8);
      }
      rem -= l;
    }
    i += m;
    lit = i;
  }
  literal(lit, n);
  return p;
}

// LZ4 block encoder (the format LZ4_compress_default writes): greedy matches over a 4-byte
// hash, offsets < 64 KiB; the last match starts >= 12 bytes before the end and the last 5 bytes
// are literals, as the format's end rules require. Returns the length.
size_t lz4_encode(const uint8_t* s, size_t n, uint8_t* o) {
  size_t p = 0;
  auto put_len = [&](size_t v) {
    for (; v >= 255; v -= 255) o[p++] = 255;
    o[p++] = (uint8_t)v;
  };
  auto sequence = [&](size_t lo, size_t hi, size_t off, size_t m) {
    const size_t ll = hi - lo, mc = m ? m - 4 : 0;
    o[p++] = (uint8_t)((ll >= 15 ? 15 : ll) << 4 | (m ? (mc >= 15 ? 15 : mc) : 0));
    if (ll >= 15) put_len(ll - 15);
    std::memcpy(o + p, s + lo, ll);
    p += ll;
    if (!m) return;
    o[p++] = (uint8_t)off;
    o[p++] = (uint8_t)(off >> 8);
    if (mc >= 15) put_len(mc - 15);
  };
  constexpr int kBits = 13;
  thread_local std::vector<int32_t> table(1 << kBits);
  std::fill(table.begin(), table.end(), -1);
  const size_t mflimit = n > 12 ? n - 12 : 0, matchlimit = n > 5 ? n - 5 : 0;
  size_t anchor = 0, i = 0;
  while (i + 4 <= n && i < mflimit) {
    uint32_t w;
    std::memcpy(&w, s + i, 4);
    const uint32_t h = (w * 2654435761u) >> (32 - kBits);
    const int32_t c = table[h];
    table[h] = (int32_t)i;
    uint32_t cw;
    if (c < 0 || i - (size_t)c > 65535 || (std::memcpy(&cw, s + c, 4), cw != w)) {
      i++;
      continue;
    }
    size_t m = 4;
    while (i + m < matchlimit && s[c + m] == s[i + m]) m++;
    sequence(anchor, i, i - (size_t)c, m);
    i += m;
    anchor = i;
  }
  sequence(anchor, n, 0, 0);
  return p;
}

}  // namespace

extern "C" {

int tpz_lz4_encode_blocks(const uint8_t* src, const uint64_t* ext, uint64_t n_blocks,
                          uint8_t* out, uint64_t out_cap, uint64_t* out_ext, uint64_t* out_len) {
  if (!src || !ext || !out || !out_ext || !out_len) return TPZ_ERR_INVALID_ARG;
  uint64_t o = 0;
  for (uint64_t b = 0; b < n_blocks; b++) {
    const uint8_t* blk = src + ext[b];
    const uint64_t len = ext[b + 1] - ext[b];
    out_ext[b] = o;
    if (len == 0 || blk[len - 1] != 1 || len - 1 > 0x7E000000ull) {  // re-encode Uncompress only
      if (o + len > out_cap) return TPZ_ERR_NOMEM;
      std::memcpy(out + o, blk, len);
      o += len;
      continue;
    }
    if (o + 32 + len + len / 255 > out_cap) return TPZ_ERR_NOMEM;
    const uint64_t body = len - 1;                          // payload | crc, before the tag
    for (int k = 0; k < 4; k++) out[o++] = (uint8_t)(body >> (8 * k));  // prepend_size (LE)
    o += lz4_encode(blk, body, out + o);
    out[o++] = 3;                                           // compress.rs:75 Lz4 tag
  }
  out_ext[n_blocks] = o;
  *out_len = o;
  return TPZ_SUCCESS;
}

int tpz_snappy_encode_blocks(const uint8_t* src, const uint64_t* ext, uint64_t n_blocks,
                             uint8_t* out, uint64_t out_cap, uint64_t* out_ext,
                             uint64_t* out_len) {
  if (!src || !ext || !out || !out_ext || !out_len) return TPZ_ERR_INVALID_ARG;
  uint64_t o = 0;
  for (uint64_t b = 0; b < n_blocks; b++) {
    const uint8_t* blk = src + ext[b];
    const uint64_t len = ext[b + 1] - ext[b];
    out_ext[b] = o;
    if (len == 0 || blk[len - 1] != 1) {  // only Uncompress blocks are re-encoded
      if (o + len > out_cap) return TPZ_ERR_NOMEM;
      std::memcpy(out + o, blk, len);
      o += len;
      continue;
    }
    if (o + 32 + 2 * len > out_cap) return TPZ_ERR_NOMEM;
    o += snappy_encode(blk, len - 1, out + o);  // payload | crc, before the codec tag
    out[o++] = 2;                                  // compress.rs:69 Snappy tag
  }
  out_ext[n_blocks] = o;
  *out_len = o;
  return TPZ_SUCCESS;
}

uint32_t tpz_host_crc32(const uint8_t* p, uint64_t n) { return crc()(p, (size_t)n); }

int tpz_build_blocks(const uint8_t* keys, const uint64_t* kpos, const uint8_t* vals,
                     const uint64_t* vpos, uint64_t n_entries, uint32_t block_size,
                     uint8_t* out, uint64_t out_cap, uint64_t* ext, uint64_t ext_cap,
                     uint64_t* n_blocks, uint64_t* out_len) {
  if (!kpos || !vpos || !out || !ext || !n_blocks || !out_len) return TPZ_ERR_INVALID_ARG;
  uint64_t o = 0, nb = 0, e = 0;
  while (e < n_entries) {
    // BlockBuilder::add fill rule (builder.rs:32): encode_len + size + 2 > target => full.
    uint64_t size = 0, first = e;
    while (e < n_entries) {
      const uint64_t kl = kpos[e + 1] - kpos[e], vl = vpos[e + 1] - vpos[e];
      if (kl == 0) return TPZ_ERR_INVALID_ARG;  // builder.rs:27 "key must not be empty"
      const uint64_t enc = 4 + kl + vl;
      if (enc + size + 2 > block_size) break;
      size += enc;
      e++;
    }
    const uint64_t n = e - first;
    if (n == 0) return TPZ_ERR_INVALID_ARG;  // entry larger than a block: the reference recurses forever
    const uint64_t blen = 2 + 2 * n + size + 4 + 1;
    if (nb + 1 >= ext_cap || o + blen > out_cap) return TPZ_ERR_NOMEM;
    uint8_t* b = out + o;
    put16(b, (uint32_t)n);  // block.rs:35
    uint8_t* d = b + 2 + 2 * n;
    uint64_t off = 0;
    for (uint64_t i = 0; i < n; i++) {
      const uint64_t x = first + i;
      const uint64_t kl = kpos[x + 1] - kpos[x], vl = vpos[x + 1] - vpos[x];
      put16(b + 2 + 2 * i, (uint32_t)off);  // builder.rs:37 (as u16)
      put16(d + off, (uint32_t)kl);          // Entry::encode builder.rs:76-79
      std::memcpy(d + off + 2, keys + kpos[x], kl);
      put16(d + off + 2 + kl, (uint32_t)vl);
      std::memcpy(d + off + 4 + kl, vals + vpos[x], vl);
      off += 4 + kl + vl;
    }
    const uint64_t plen = 2 + 2 * n + size;
    put32(b + plen, crc()(b, plen));  // block.rs:41-42
    b[plen + 4] = 1;                  // compress.rs:87 Uncompress tag
    ext[nb++] = o;
    o += blen;
  }
  ext[nb] = o;
  *n_blocks = nb;
  *out_len = o;
  return TPZ_SUCCESS;
}

}  // extern "C"
