// tpz_host_builder.cpp — host write side: BlockBuilder + SsTableBuilder block packing.
//
// Restates src/block/builder.rs:26-85 (fill rule, Entry::encode), src/block.rs:31-44
// (Block::encode: u16 n | u16 off[n] | entries | u32 crc32 | codec tag) and
// src/table/builder.rs:49-85 (SsTableBuilder::add / block_build: one block after another,
// back to back) for the Uncompress codec (src/block/compress.rs:85-89). It produces SST data
// regions for bench.py and for the table facade; it is not on the decode path.
#include <cstdint>
#include <cstring>

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

}  // namespace

extern "C" {

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
