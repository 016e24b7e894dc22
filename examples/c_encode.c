/*
 * c_encode.c — a plain C consumer of the device write side (include/tpz_gpu.h): sorted entries
 * in HBM become SST data-region blocks, what SsTableBuilder::add + block_build writes
 * (src/table/builder.rs:49-85) with CompressOptions::Uncompress.
 *
 *   1. make n entries on the host (keys: 8-byte big-endian counter + 1..24 random bytes;
 *      values: 0..300 random bytes, fewer for small blocks), upload keys/values and offsets;
 *   2. tpz_plan_blocks (the fill rule's block cuts) + tpz_encode_blocks (Block::encode, CRC, tag);
 *   3. compare the region and the block offsets with tpz_build_blocks (the host restatement),
 *      then decode the device region with tpz_decode_blocks and check every block is OK with
 *      the planned entry count;
 *   4. an entry with an empty key must be refused with its index (builder.rs:27);
 *   5. the region in the flat layout (tpz_flat_layout + tpz_decode_blocks_flat): the key and
 *      value columns equal the entries' keys and values back to back;
 *   6. compaction output with snappy on the device (tpz_compress_blocks), back through the
 *      codec step to the same bytes.
 * Prints "ok <entries> <blocks>" and exits 0, or the first mismatch and exits 1.
 * Usage: c_encode [n_entries] [block_size]
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "tpz_gpu.h"

#define CHECK_HIP(x)                                                        \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
      return 1;                                                             \
    }                                                                       \
  } while (0)
#define CHECK_TPZ(x)                                                        \
  do {                                                                      \
    int e_ = (x);                                                           \
    if (e_ != TPZ_SUCCESS) {                                                \
      fprintf(stderr, "%s: %d %s\n", #x, e_, tpz_last_error());             \
      return 1;                                                             \
    }                                                                       \
  } while (0)

static uint64_t splitmix(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)strtoul(argv[1], NULL, 10) : 50000;
  const uint32_t block_size = argc > 2 ? (uint32_t)strtoul(argv[2], NULL, 10) : 4096;
  uint64_t seed = 0x5EED0005ull;
  uint64_t* kpos = malloc(((size_t)n + 1) * 8);
  uint64_t* vpos = malloc(((size_t)n + 1) * 8);
  /* every entry fits a block: 4 + 32 (longest key) + vmax <= block_size - 2 */
  const uint64_t vmax = block_size >= 338 ? 300 : (block_size > 38 ? block_size - 38 : 0);
  kpos[0] = vpos[0] = 0;
  for (uint32_t i = 0; i < n; i++) {
    kpos[i + 1] = kpos[i] + 8 + 1 + splitmix(&seed) % 24;
    vpos[i + 1] = vpos[i] + splitmix(&seed) % (vmax + 1);
  }
  uint8_t* keys = malloc(kpos[n] + 1);
  uint8_t* vals = malloc(vpos[n] + 1);
  for (uint32_t i = 0; i < n; i++) {
    uint8_t* k = keys + kpos[i];
    for (int b = 0; b < 8; b++) k[b] = (uint8_t)((uint64_t)i >> (56 - 8 * b));   /* sorted */
    for (uint64_t b = 8; b < kpos[i + 1] - kpos[i]; b++) k[b] = (uint8_t)splitmix(&seed);
  }
  for (uint64_t b = 0; b < vpos[n]; b++) vals[b] = (uint8_t)splitmix(&seed);

  /* the host restatement's region (tpz_build_blocks) */
  const uint64_t cap = kpos[n] + vpos[n] + 13ull * n + 64;
  uint8_t* ref = malloc(cap);
  uint64_t* ref_ext = malloc(((size_t)n + 2) * 8);
  uint64_t ref_nb = 0, ref_len = 0;
  CHECK_TPZ(tpz_build_blocks(keys, kpos, vals, vpos, n, block_size, ref, cap, ref_ext, n + 2,
                             &ref_nb, &ref_len));

  tpz_ctx* ctx = NULL;
  CHECK_TPZ(tpz_ctx_create(0, &ctx));
  hipStream_t st;
  CHECK_HIP(hipStreamCreate(&st));
  uint8_t *d_keys, *d_vals, *d_out;
  uint64_t *d_kpos, *d_vpos, *d_ext;
  uint32_t* d_first;
  CHECK_HIP(hipMalloc((void**)&d_keys, kpos[n] + 16));
  CHECK_HIP(hipMalloc((void**)&d_vals, vpos[n] + 16));
  CHECK_HIP(hipMalloc((void**)&d_kpos, ((size_t)n + 1) * 8));
  CHECK_HIP(hipMalloc((void**)&d_vpos, ((size_t)n + 1) * 8));
  CHECK_HIP(hipMalloc((void**)&d_first, ((size_t)n + 1) * 4));
  CHECK_HIP(hipMalloc((void**)&d_ext, ((size_t)n + 1) * 8));
  CHECK_HIP(hipMemcpy(d_keys, keys, kpos[n], hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(d_vals, vals, vpos[n], hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(d_kpos, kpos, ((size_t)n + 1) * 8, hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(d_vpos, vpos, ((size_t)n + 1) * 8, hipMemcpyHostToDevice));

  tpz_entries ent = {d_keys, d_kpos, d_vals, d_vpos, n, kpos[n], vpos[n]};
  uint32_t nb = 0;
  uint64_t bad = 0;
  CHECK_TPZ(tpz_plan_blocks(ctx, &ent, block_size, d_first, d_ext, &nb, &bad, st));
  if (nb != ref_nb) {
    printf("n_blocks %u != %llu\n", nb, (unsigned long long)ref_nb);
    return 1;
  }
  uint64_t* ext = malloc(((size_t)nb + 1) * 8);
  uint32_t* first = malloc(((size_t)nb + 1) * 4);
  CHECK_HIP(hipMemcpy(ext, d_ext, ((size_t)nb + 1) * 8, hipMemcpyDeviceToHost));
  CHECK_HIP(hipMemcpy(first, d_first, ((size_t)nb + 1) * 4, hipMemcpyDeviceToHost));
  for (uint32_t b = 0; b <= nb; b++)
    if (ext[b] != ref_ext[b]) {
      printf("ext[%u] %llu != %llu\n", b, (unsigned long long)ext[b], (unsigned long long)ref_ext[b]);
      return 1;
    }
  CHECK_HIP(hipMalloc((void**)&d_out, ext[nb] + 16));
  CHECK_TPZ(tpz_encode_blocks(ctx, &ent, d_first, d_ext, nb, d_out, st));
  CHECK_HIP(hipStreamSynchronize(st));
  uint8_t* out = malloc(ext[nb] + 1);
  CHECK_HIP(hipMemcpy(out, d_out, ext[nb], hipMemcpyDeviceToHost));
  if (memcmp(out, ref, ext[nb]) != 0) {
    for (uint64_t i = 0; i < ext[nb]; i++)
      if (out[i] != ref[i]) {
        printf("byte %llu differs\n", (unsigned long long)i);
        return 1;
      }
  }

  /* the device region decodes: every block OK with its planned entry count */
  tpz_batch batch = {d_out, d_ext, nb, ext[nb]};
  const uint64_t dcap = tpz_data_capacity(ext[nb], nb), ecap = tpz_entry_capacity(ext[nb], nb);
  tpz_columns cols;
  memset(&cols, 0, sizeof cols);
  CHECK_HIP(hipMalloc((void**)&cols.d_data, dcap));
  CHECK_HIP(hipMalloc((void**)&cols.d_ends, 2 * ecap * 4));
  CHECK_HIP(hipMalloc((void**)&cols.d_count, (size_t)nb * 4));
  CHECK_HIP(hipMalloc((void**)&cols.d_status, nb));
  CHECK_HIP(hipMalloc((void**)&cols.d_crc, (size_t)nb * 4));
  CHECK_HIP(hipMalloc((void**)&cols.d_spill_off, (size_t)nb * 8));
  CHECK_HIP(hipMalloc((void**)&cols.d_spill_used, 8));
  CHECK_TPZ(tpz_decode_blocks(ctx, &batch, &cols, st));
  CHECK_HIP(hipStreamSynchronize(st));
  uint8_t* status = malloc(nb);
  uint32_t* count = malloc((size_t)nb * 4);
  CHECK_HIP(hipMemcpy(status, cols.d_status, nb, hipMemcpyDeviceToHost));
  CHECK_HIP(hipMemcpy(count, cols.d_count, (size_t)nb * 4, hipMemcpyDeviceToHost));
  for (uint32_t b = 0; b < nb; b++)
    if (status[b] != TPZ_BLOCK_OK || count[b] != first[b + 1] - first[b]) {
      printf("block %u: status %u count %u, planned %u entries\n", b, status[b], count[b],
             first[b + 1] - first[b]);
      return 1;
    }

  /* 5. the same region into the flat layout (tpz_flat_layout + tpz_decode_blocks_flat): the key
   *    column must be the entries' keys back to back, the value column their values, and every
   *    {kend, vend} pair the entry's end within its block */
  {
    uint64_t* d_fl;
    const uint64_t st1 = (uint64_t)nb + 1;
    CHECK_HIP(hipMalloc((void**)&d_fl, 3 * st1 * 8));
    CHECK_TPZ(tpz_flat_layout(ctx, &batch, d_fl, st));
    uint64_t* fl = malloc(3 * st1 * 8);
    CHECK_HIP(hipStreamSynchronize(st));
    CHECK_HIP(hipMemcpy(fl, d_fl, 3 * st1 * 8, hipMemcpyDeviceToHost));
    if (fl[nb] != n || fl[st1 + nb] != kpos[n] || fl[2 * st1 + nb] != vpos[n]) {
      printf("flat totals %llu %llu %llu\n", (unsigned long long)fl[nb],
             (unsigned long long)fl[st1 + nb], (unsigned long long)fl[2 * st1 + nb]);
      return 1;
    }
    tpz_flat_columns fc;
    memset(&fc, 0, sizeof fc);
    CHECK_HIP(hipMalloc((void**)&fc.d_keys, kpos[n] + 16));
    CHECK_HIP(hipMalloc((void**)&fc.d_values, vpos[n] + 16));
    CHECK_HIP(hipMalloc((void**)&fc.d_ends, (size_t)n * 8 + 8));
    fc.d_first = d_fl;
    fc.d_count = cols.d_count;
    fc.d_status = cols.d_status;
    fc.d_crc = cols.d_crc;
    fc.d_spill_off = cols.d_spill_off;
    fc.d_spill_used = cols.d_spill_used;
    CHECK_TPZ(tpz_decode_blocks_flat(ctx, &batch, &fc, st));
    CHECK_TPZ(tpz_decode_check(ctx, st));
    uint8_t* fk = malloc(kpos[n] + 1);
    uint8_t* fv = malloc(vpos[n] + 1);
    uint32_t* fe = malloc((size_t)n * 8 + 8);
    CHECK_HIP(hipMemcpy(fk, fc.d_keys, kpos[n], hipMemcpyDeviceToHost));
    CHECK_HIP(hipMemcpy(fv, fc.d_values, vpos[n], hipMemcpyDeviceToHost));
    CHECK_HIP(hipMemcpy(fe, fc.d_ends, (size_t)n * 8, hipMemcpyDeviceToHost));
    CHECK_HIP(hipMemcpy(status, cols.d_status, nb, hipMemcpyDeviceToHost));
    for (uint32_t b = 0; b < nb; b++)
      if (status[b] != TPZ_BLOCK_OK) {
        printf("flat: block %u status %u\n", b, status[b]);
        return 1;
      }
    if (memcmp(fk, keys, kpos[n]) != 0 || memcmp(fv, vals, vpos[n]) != 0) {
      printf("flat columns differ from the entries\n");
      return 1;
    }
    for (uint32_t b = 0; b < nb; b++)
      for (uint32_t e = first[b]; e < first[b + 1]; e++)
        if (fe[2 * e] != kpos[e + 1] - kpos[first[b]] || fe[2 * e + 1] != vpos[e + 1] - vpos[first[b]]) {
          printf("flat: entry %u ends %u %u\n", e, fe[2 * e], fe[2 * e + 1]);
          return 1;
        }
    free(fk);
    free(fv);
    free(fe);
    free(fl);
  }

  /* 6. compaction output with the default codec: the region to snappy blocks on the device
   *    (tpz_compress_blocks), back through the codec step and the decode: every block OK with its
   *    planned count */
  {
    const uint64_t ccap = tpz_layout_compress_bound(ext[nb], nb);
    uint8_t *d_c, *d_u;
    uint64_t *d_cext, *d_uext;
    CHECK_HIP(hipMalloc((void**)&d_c, ccap));
    CHECK_HIP(hipMalloc((void**)&d_cext, ((size_t)nb + 1) * 8));
    CHECK_TPZ(tpz_compress_blocks(ctx, &batch, 2, d_c, d_cext, st));
    uint64_t* cext = malloc(((size_t)nb + 1) * 8);
    CHECK_HIP(hipStreamSynchronize(st));
    CHECK_HIP(hipMemcpy(cext, d_cext, ((size_t)nb + 1) * 8, hipMemcpyDeviceToHost));
    tpz_batch cb = {d_c, d_cext, nb, cext[nb]};
    uint64_t* sz = malloc(((size_t)nb + 1) * 8);
    uint64_t* d_sz;
    CHECK_HIP(hipMalloc((void**)&d_sz, (size_t)nb * 8));
    CHECK_TPZ(tpz_decompressed_sizes(ctx, &cb, d_sz, st));
    CHECK_HIP(hipStreamSynchronize(st));
    CHECK_HIP(hipMemcpy(sz + 1, d_sz, (size_t)nb * 8, hipMemcpyDeviceToHost));
    sz[0] = 0;
    for (uint32_t b = 0; b < nb; b++) sz[b + 1] += sz[b];
    if (sz[nb] != ext[nb]) {
      printf("decompressed size %llu != %llu\n", (unsigned long long)sz[nb], (unsigned long long)ext[nb]);
      return 1;
    }
    CHECK_HIP(hipMalloc((void**)&d_u, sz[nb] + 16));
    CHECK_HIP(hipMalloc((void**)&d_uext, ((size_t)nb + 1) * 8));
    CHECK_HIP(hipMemcpy(d_uext, sz, ((size_t)nb + 1) * 8, hipMemcpyHostToDevice));
    CHECK_TPZ(tpz_decompress_blocks(ctx, &cb, d_u, d_uext, cols.d_status, st));
    CHECK_HIP(hipStreamSynchronize(st));
    uint8_t* u = malloc(sz[nb] + 1);
    CHECK_HIP(hipMemcpy(u, d_u, sz[nb], hipMemcpyDeviceToHost));
    if (memcmp(u, out, ext[nb]) != 0) {
      printf("snappy round trip differs (%llu compressed bytes)\n", (unsigned long long)cext[nb]);
      return 1;
    }
    free(u);
    free(sz);
    free(cext);
  }

  /* an empty key is refused with its index (builder.rs:27 asserts) */
  uint64_t kpos2[3] = {0, 3, 3};
  uint64_t vpos2[3] = {0, 1, 2};
  CHECK_HIP(hipMemcpy(d_kpos, kpos2, sizeof kpos2, hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(d_vpos, vpos2, sizeof vpos2, hipMemcpyHostToDevice));
  tpz_entries ent2 = {d_keys, d_kpos, d_vals, d_vpos, 2, kpos[n], vpos[n]};
  if (tpz_plan_blocks(ctx, &ent2, block_size, d_first, d_ext, &nb, &bad, st) != TPZ_ERR_INVALID_ARG ||
      bad != 1) {
    printf("empty key not refused (bad %llu)\n", (unsigned long long)bad);
    return 1;
  }

  printf("ok %u %llu\n", n, (unsigned long long)ref_nb);
  tpz_ctx_destroy(ctx);
  return 0;
}
