// tpz_xxh3.h — XXH3_64bits (seed 0, default secret), host and device.
//
// The reference hashes keys for its bloom filter with xxhash_rust::xxh3::xxh3_64 (xxhash-rust
// 0.8.5, Cargo.toml:25-27; call sites src/table.rs:114-119 may_contain and the builder's
// from_keys). Restated from the published XXH3 algorithm (xxHash 0.8 spec): the 0-16, 17-128,
// 129-240 byte paths and the long-input path (8 accumulators, 64-byte stripes, a scramble per
// 1 KiB block). Pinned against Python's xxhash 3.8.1 (xxh3_64) in tests/test_abi.py.
#pragma once

#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define TPZ_HD __host__ __device__
#else
#define TPZ_HD
#endif

namespace tpz {
namespace xxh3 {

constexpr uint64_t kP32_1 = 0x9E3779B1ull, kP32_2 = 0x85EBCA77ull, kP32_3 = 0xC2B2AE3Dull;
constexpr uint64_t kP64_1 = 0x9E3779B185EBCA87ull, kP64_2 = 0xC2B2AE3D27D4EB4Full;
constexpr uint64_t kP64_3 = 0x165667B19E3779F9ull, kP64_4 = 0x85EBCA77C2B2AE63ull;
constexpr uint64_t kP64_5 = 0x27D4EB2F165667C5ull;
constexpr uint64_t kMx1 = 0x165667919E3779F9ull, kMx2 = 0x9FB21C651E98DF25ull;

// The default 192-byte secret (kSecret of the spec), as little-endian u64 words.
TPZ_HD inline uint64_t secret64(uint32_t off) {
  // byte offsets used by XXH3 are not all 8-aligned: read bytes
  constexpr uint8_t k[192] = {
      0xb8, 0xfe, 0x6c, 0x39, 0x23, 0xa4, 0x4b, 0xbe, 0x7c, 0x01, 0x81, 0x2c, 0xf7, 0x21, 0xad,
      0x1c, 0xde, 0xd4, 0x6d, 0xe9, 0x83, 0x90, 0x97, 0xdb, 0x72, 0x40, 0xa4, 0xa4, 0xb7, 0xb3,
      0x67, 0x1f, 0xcb, 0x79, 0xe6, 0x4e, 0xcc, 0xc0, 0xe5, 0x78, 0x82, 0x5a, 0xd0, 0x7d, 0xcc,
      0xff, 0x72, 0x21, 0xb8, 0x08, 0x46, 0x74, 0xf7, 0x43, 0x24, 0x8e, 0xe0, 0x35, 0x90, 0xe6,
      0x81, 0x3a, 0x26, 0x4c, 0x3c, 0x28, 0x52, 0xbb, 0x91, 0xc3, 0x00, 0xcb, 0x88, 0xd0, 0x65,
      0x8b, 0x1b, 0x53, 0x2e, 0xa3, 0x71, 0x64, 0x48, 0x97, 0xa2, 0x0d, 0xf9, 0x4e, 0x38, 0x19,
      0xef, 0x46, 0xa9, 0xde, 0xac, 0xd8, 0xa8, 0xfa, 0x76, 0x3f, 0xe3, 0x9c, 0x34, 0x3f, 0xf9,
      0xdc, 0xbb, 0xc7, 0xc7, 0x0b, 0x4f, 0x1d, 0x8a, 0x51, 0xe0, 0x4b, 0xcd, 0xb4, 0x59, 0x31,
      0xc8, 0x9f, 0x7e, 0xc9, 0xd9, 0x78, 0x73, 0x64, 0xea, 0xc5, 0xac, 0x83, 0x34, 0xd3, 0xeb,
      0xc3, 0xc5, 0x81, 0xa0, 0xff, 0xfa, 0x13, 0x63, 0xeb, 0x17, 0x0d, 0xdd, 0x51, 0xb7, 0xf0,
      0xda, 0x49, 0xd3, 0x16, 0x55, 0x26, 0x29, 0xd4, 0x68, 0x9e, 0x2b, 0x16, 0xbe, 0x58, 0x7d,
      0x47, 0xa1, 0xfc, 0x8f, 0xf8, 0xb8, 0xd1, 0x7a, 0xd0, 0x31, 0xce, 0x45, 0xcb, 0x3a, 0x8f,
      0x95, 0x16, 0x04, 0x28, 0xaf, 0xd7, 0xfb, 0xca, 0xbb, 0x4b, 0x40, 0x7e};
  uint64_t v = 0;
  for (int i = 7; i >= 0; i--) v = (v << 8) | k[off + i];
  return v;
}
TPZ_HD inline uint32_t secret32(uint32_t off) { return (uint32_t)secret64(off); }

// Little-endian reads at any alignment: one (unaligned) dwordx2 / dword load on gfx950 instead of
// eight / four byte loads (TPZ_XXH3_BYTEREADS keeps the byte loads, for A/B builds).
TPZ_HD inline uint64_t rd64(const uint8_t* p) {
#if defined(TPZ_XXH3_BYTEREADS)
  uint64_t v = 0;
  for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
  return v;
#else
  uint64_t v;
  memcpy(&v, p, 8);
  return v;
#endif
}
TPZ_HD inline uint32_t rd32(const uint8_t* p) {
#if defined(TPZ_XXH3_BYTEREADS)
  return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
#else
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
#endif
}
TPZ_HD inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
TPZ_HD inline uint64_t swap64(uint64_t x) {
  x = ((x & 0x00FF00FF00FF00FFull) << 8) | ((x >> 8) & 0x00FF00FF00FF00FFull);
  x = ((x & 0x0000FFFF0000FFFFull) << 16) | ((x >> 16) & 0x0000FFFF0000FFFFull);
  return (x << 32) | (x >> 32);
}
TPZ_HD inline uint64_t mul128_fold64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (a * b) ^ __umul64hi(a, b);
#else
  const unsigned __int128 p = (unsigned __int128)a * b;
  return (uint64_t)p ^ (uint64_t)(p >> 64);
#endif
}
TPZ_HD inline uint64_t avalanche(uint64_t h) {
  h ^= h >> 37;
  h *= kMx1;
  return h ^ (h >> 32);
}
TPZ_HD inline uint64_t xxh64_avalanche(uint64_t h) {
  h ^= h >> 33;
  h *= kP64_2;
  h ^= h >> 29;
  h *= kP64_3;
  return h ^ (h >> 32);
}
TPZ_HD inline uint64_t rrmxmx(uint64_t h, uint64_t len) {
  h ^= rotl64(h, 49) ^ rotl64(h, 24);
  h *= kMx2;
  h ^= (h >> 35) + len;
  h *= kMx2;
  return h ^ (h >> 28);
}
TPZ_HD inline uint64_t mix16(const uint8_t* in, uint32_t s) {
  return mul128_fold64(rd64(in) ^ secret64(s), rd64(in + 8) ^ secret64(s + 8));
}
TPZ_HD inline void accumulate512(uint64_t* acc, const uint8_t* in, uint32_t s) {
  for (int i = 0; i < 8; i++) {
    const uint64_t v = rd64(in + 8 * i), k = v ^ secret64(s + 8 * i);
    acc[i ^ 1] += v;
    acc[i] += (uint64_t)(uint32_t)k * (k >> 32);
  }
}
TPZ_HD inline void scramble(uint64_t* acc, uint32_t s) {
  for (int i = 0; i < 8; i++) {
    uint64_t a = acc[i];
    a ^= a >> 47;
    a ^= secret64(s + 8 * i);
    acc[i] = a * kP32_1;
  }
}

TPZ_HD inline uint64_t hash64(const uint8_t* in, uint64_t len) {
  if (len <= 16) {
    if (len > 8) {
      const uint64_t lo = rd64(in) ^ (secret64(24) ^ secret64(32));
      const uint64_t hi = rd64(in + len - 8) ^ (secret64(40) ^ secret64(48));
      return avalanche(len + swap64(lo) + hi + mul128_fold64(lo, hi));
    }
    if (len >= 4) {
      const uint64_t v = rd32(in + len - 4) + ((uint64_t)rd32(in) << 32);
      return rrmxmx(v ^ (secret64(8) ^ secret64(16)), len);
    }
    if (len > 0) {
      const uint32_t c = ((uint32_t)in[0] << 16) | ((uint32_t)in[len >> 1] << 24) |
                         (uint32_t)in[len - 1] | ((uint32_t)len << 8);
      return xxh64_avalanche((uint64_t)c ^ (uint64_t)(secret32(0) ^ secret32(4)));
    }
    return xxh64_avalanche(secret64(56) ^ secret64(64));
  }
  if (len <= 128) {
    uint64_t acc = len * kP64_1;
    if (len > 32) {
      if (len > 64) {
        if (len > 96) {
          acc += mix16(in + 48, 96);
          acc += mix16(in + len - 64, 112);
        }
        acc += mix16(in + 32, 64);
        acc += mix16(in + len - 48, 80);
      }
      acc += mix16(in + 16, 32);
      acc += mix16(in + len - 32, 48);
    }
    acc += mix16(in, 0);
    acc += mix16(in + len - 16, 16);
    return avalanche(acc);
  }
  if (len <= 240) {
    uint64_t acc = len * kP64_1;
    const uint32_t rounds = (uint32_t)(len / 16);
    for (uint32_t i = 0; i < 8; i++) acc += mix16(in + 16 * i, 16 * i);
    acc = avalanche(acc);
    for (uint32_t i = 8; i < rounds; i++) acc += mix16(in + 16 * i, 16 * (i - 8) + 3);
    acc += mix16(in + len - 16, 136 - 17);
    return avalanche(acc);
  }
  uint64_t acc[8] = {kP32_3, kP64_1, kP64_2, kP64_3, kP64_4, kP32_2, kP64_5, kP32_1};
  constexpr uint32_t kStripes = (192 - 64) / 8, kBlock = 64 * kStripes;
  const uint64_t nb = (len - 1) / kBlock;
  for (uint64_t b = 0; b < nb; b++) {
    for (uint32_t n = 0; n < kStripes; n++) accumulate512(acc, in + b * kBlock + 64 * n, 8 * n);
    scramble(acc, 192 - 64);
  }
  const uint32_t ns = (uint32_t)(((len - 1) - kBlock * nb) / 64);
  for (uint32_t n = 0; n < ns; n++) accumulate512(acc, in + nb * kBlock + 64 * n, 8 * n);
  accumulate512(acc, in + len - 64, 192 - 64 - 7);
  uint64_t r = len * kP64_1;
  for (int i = 0; i < 4; i++)
    r += mul128_fold64(acc[2 * i] ^ secret64(11 + 16 * i), acc[2 * i + 1] ^ secret64(11 + 16 * i + 8));
  return avalanche(r);
}

}  // namespace xxh3
}  // namespace tpz
