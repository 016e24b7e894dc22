/*
 * c_abi_decode.c — a plain C consumer of include/tpz_gpu.h (no Python, no torch): what a
 * topazdb host binding does through the C ABI.
 *
 *   1. build N Uncompress blocks of BlockBuilder entries on the host (tpz_build_blocks,
 *      src/table/builder.rs:49-85);
 *   2. copy them to HBM, decode + verify them on the GPU (tpz_decode_blocks);
 *   3. check every block's status and CRC (against tpz_host_crc32 over the payload) and every
 *      key and value against what was built, reading the slotted layout with the header's
 *      layout helpers; then the whole-range CRC (tpz_crc32_ranges) of each block's payload.
 * Prints "ok <blocks> <entries>" and exits 0, or prints the first mismatch and exits 1.
 *
 * Build (tests/test_abi.py compiles it with gcc; tests/test_gpu_c_abi.py runs it):
 *   gcc -std=c11 -O2 -D__HIP_PLATFORM_AMD__ -I include -I /opt/rocm/include \
 *       examples/c_abi_decode.c -o c_abi_decode -L topazdb_amd -ltpz_gpu \
 *       -L /opt/rocm/lib -lamdhip64 -Wl,-rpath,$PWD/topazdb_amd -Wl,-rpath,/opt/rocm/lib
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
  const uint64_t n_entries = argc > 1 ? strtoull(argv[1], NULL, 10) : 20000;
  /* entries: 16-B keys (8-B big-endian counter + 8 random bytes), 1..200-B values */
  uint64_t seed = 0x5EED0C0Dull;
  uint64_t* kpos = malloc((n_entries + 1) * sizeof(uint64_t));
  uint64_t* vpos = malloc((n_entries + 1) * sizeof(uint64_t));
  uint8_t* keys = malloc(16 * n_entries);
  uint8_t* vals = malloc(200 * n_entries + 1);
  kpos[0] = vpos[0] = 0;
  for (uint64_t e = 0; e < n_entries; e++) {
    for (int i = 0; i < 8; i++) keys[16 * e + i] = (uint8_t)(e >> (56 - 8 * i));
    const uint64_t r = splitmix(&seed);
    memcpy(keys + 16 * e + 8, &r, 8);
    kpos[e + 1] = 16 * (e + 1);
    const uint64_t vl = 1 + splitmix(&seed) % 200;
    for (uint64_t i = 0; i < vl; i++) vals[vpos[e] + i] = (uint8_t)splitmix(&seed);
    vpos[e + 1] = vpos[e] + vl;
  }
  const uint64_t cap = 2 * (kpos[n_entries] + vpos[n_entries]) + 1024;
  uint8_t* blocks = malloc(cap);
  uint64_t* ext = malloc((n_entries + 2) * sizeof(uint64_t));
  uint64_t nb = 0, len = 0;
  CHECK_TPZ(tpz_build_blocks(keys, kpos, vals, vpos, n_entries, 4096, blocks, cap, ext,
                             n_entries + 2, &nb, &len));

  tpz_ctx* ctx = NULL;
  CHECK_TPZ(tpz_ctx_create(0, &ctx));
  hipStream_t stream;
  CHECK_HIP(hipStreamCreate(&stream));
  uint8_t* d_src;
  uint64_t* d_ext;
  CHECK_HIP(hipMalloc((void**)&d_src, len));
  CHECK_HIP(hipMalloc((void**)&d_ext, (nb + 1) * sizeof(uint64_t)));
  CHECK_HIP(hipMemcpy(d_src, blocks, len, hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(d_ext, ext, (nb + 1) * sizeof(uint64_t), hipMemcpyHostToDevice));

  const uint64_t dcap = tpz_data_capacity(len, nb), ecap = tpz_entry_capacity(len, nb);
  tpz_columns cols;
  CHECK_HIP(hipMalloc((void**)&cols.d_data, dcap));
  CHECK_HIP(hipMalloc((void**)&cols.d_ends, 2 * ecap * sizeof(uint32_t)));
  CHECK_HIP(hipMalloc((void**)&cols.d_count, nb * sizeof(uint32_t)));
  CHECK_HIP(hipMalloc((void**)&cols.d_status, nb));
  CHECK_HIP(hipMalloc((void**)&cols.d_crc, nb * sizeof(uint32_t)));
  /* BlockBuilder output never spills (include/tpz_gpu.h): no arena, but the per-block offsets
   * and the used-bytes word are always given */
  cols.d_spill = NULL;
  cols.spill_cap = 0;
  CHECK_HIP(hipMalloc((void**)&cols.d_spill_off, nb * sizeof(uint64_t)));
  CHECK_HIP(hipMalloc((void**)&cols.d_spill_used, sizeof(uint64_t)));
  const tpz_batch batch = {d_src, d_ext, (uint32_t)nb, len};
  CHECK_TPZ(tpz_decode_blocks(ctx, &batch, &cols, stream));

  /* the payload CRC of every block as a range batch: [ext[i], ext[i+1] - 5) */
  uint64_t* pext = malloc(2 * nb * sizeof(uint64_t));
  for (uint64_t i = 0; i < nb; i++) {
    pext[2 * i] = ext[i];
    pext[2 * i + 1] = ext[i + 1] - 5;
  }
  /* ranges must be contiguous extents: CRC each payload as its own one-range batch */
  uint32_t* d_rcrc;
  CHECK_HIP(hipMalloc((void**)&d_rcrc, nb * sizeof(uint32_t)));
  uint64_t* d_pext;
  CHECK_HIP(hipMalloc((void**)&d_pext, 2 * nb * sizeof(uint64_t)));
  CHECK_HIP(hipMemcpy(d_pext, pext, 2 * nb * sizeof(uint64_t), hipMemcpyHostToDevice));
  for (uint64_t i = 0; i < nb; i++) {
    const tpz_batch r = {d_src, d_pext + 2 * i, 1, len};
    CHECK_TPZ(tpz_crc32_ranges(ctx, &r, d_rcrc + i, stream));
  }
  CHECK_HIP(hipStreamSynchronize(stream));

  uint8_t* data = malloc(dcap);
  uint32_t* ends = malloc(2 * ecap * sizeof(uint32_t));
  uint32_t* count = malloc(nb * sizeof(uint32_t));
  uint8_t* status = malloc(nb);
  uint32_t* crc = malloc(nb * sizeof(uint32_t));
  uint32_t* rcrc = malloc(nb * sizeof(uint32_t));
  CHECK_HIP(hipMemcpy(data, cols.d_data, dcap, hipMemcpyDeviceToHost));
  CHECK_HIP(hipMemcpy(ends, cols.d_ends, 2 * ecap * sizeof(uint32_t), hipMemcpyDeviceToHost));
  CHECK_HIP(hipMemcpy(count, cols.d_count, nb * sizeof(uint32_t), hipMemcpyDeviceToHost));
  CHECK_HIP(hipMemcpy(status, cols.d_status, nb, hipMemcpyDeviceToHost));
  CHECK_HIP(hipMemcpy(crc, cols.d_crc, nb * sizeof(uint32_t), hipMemcpyDeviceToHost));
  CHECK_HIP(hipMemcpy(rcrc, d_rcrc, nb * sizeof(uint32_t), hipMemcpyDeviceToHost));

  uint64_t e = 0;
  for (uint64_t b = 0; b < nb; b++) {
    const uint32_t want_crc = tpz_host_crc32(blocks + ext[b], ext[b + 1] - ext[b] - 5);
    if (status[b] != TPZ_BLOCK_OK || crc[b] != want_crc || rcrc[b] != want_crc) {
      printf("block %llu: status %u crc %08x range crc %08x want %08x\n", (unsigned long long)b,
             status[b], crc[b], rcrc[b], want_crc);
      return 1;
    }
    const uint64_t s = tpz_slot_base(ext[b], b), eb = tpz_entry_base(ext[b], b);
    const uint32_t n = count[b];
    const uint64_t K = n ? ends[2 * (eb + n - 1)] : 0, vs = tpz_value_start(K);
    for (uint32_t j = 0; j < n; j++, e++) {
      const uint32_t k0 = j ? ends[2 * (eb + j - 1)] : 0, k1 = ends[2 * (eb + j)];
      const uint32_t v0 = j ? ends[2 * (eb + j - 1) + 1] : 0, v1 = ends[2 * (eb + j) + 1];
      if (e >= n_entries || k1 - k0 != kpos[e + 1] - kpos[e] ||
          memcmp(data + s + k0, keys + kpos[e], k1 - k0) != 0 ||
          v1 - v0 != vpos[e + 1] - vpos[e] ||
          memcmp(data + s + vs + v0, vals + vpos[e], v1 - v0) != 0) {
        printf("block %llu entry %u differs\n", (unsigned long long)b, j);
        return 1;
      }
    }
  }
  if (e != n_entries) {
    printf("%llu of %llu entries decoded\n", (unsigned long long)e,
           (unsigned long long)n_entries);
    return 1;
  }
  printf("ok %llu %llu\n", (unsigned long long)nb, (unsigned long long)e);
  tpz_ctx_destroy(ctx);
  return 0;
}
