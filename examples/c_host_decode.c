/*
 * c_host_decode.c — a plain C consumer of tpz_decode_blocks_host (include/tpz_gpu.h): blocks in
 * host memory (what FileObject::read returns, src/table/file_object.rs:23-27) go through the
 * library's own H2D -> decode -> D2H pipeline and come back decoded into host buffers.
 *
 *   1. build Uncompress blocks of BlockBuilder entries on the host (tpz_build_blocks), corrupt
 *      one block's payload, optionally compress every block with snappy (codec 2) or lz4
 *      (codec 3) as compress::encode does (src/block/compress.rs:66-77) and append a stream
 *      the codec rejects, and append a hand-made Uncompress block whose 64 offsets all point at
 *      one 2000-byte key (the reference iterator accepts repeated offsets: it spills);
 *   2. tpz_decode_blocks_host with small chunks (several pipeline rounds);
 *   3. check every status and CRC, every key and value of the built entries (slotted h_data at
 *      the decoded extents h_dext + dense h_ends), and the spilled block's record in h_spill.
 * Prints "ok <blocks> <entries> <GiB/s>" and exits 0, or the first mismatch and exits 1.
 * Usage: c_host_decode [n_entries] [chunk_blocks] [pinned] [codec 0|2|3]
 *        c_host_decode --sst FILE [chunk_blocks]: an SST file (FileObject::open's trailer chain,
 *        src/table.rs:75-112) decoded through the pipeline; prints every entry as
 *        "<hex key> <hex value>" in SsTableIterator order, then "ok sst <blocks> <entries>".
 */
#define _POSIX_C_SOURCE 199309L
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

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

static uint32_t be32(const uint8_t* p) {
  return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}

static void hex(const uint8_t* p, size_t n) {
  static const char* d = "0123456789abcdef";
  for (size_t i = 0; i < n; i++) putchar(d[p[i] >> 4]), putchar(d[p[i] & 15]);
}

/* An SST file through tpz_decode_blocks_host: read_bloom + meta (table.rs:75-112, 49-59) give
 * the block extents (table.rs:154-161); every decoded entry is printed in iteration order. */
static int sst_mode(const char* path, uint32_t chunk) {
  FILE* f = fopen(path, "rb");
  if (!f) return 1;
  fseek(f, 0, SEEK_END);
  const long flen = ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t* file = malloc((size_t)flen);
  if (fread(file, 1, (size_t)flen, f) != (size_t)flen) return 1;
  fclose(f);
  const uint64_t size = (uint64_t)flen - 4;                 /* FileObject: CRC trailer */
  if (tpz_host_crc32(file, size) != be32(file + size)) return 1;
  const uint64_t bloom_off = be32(file + size - 4), meta_off = be32(file + bloom_off - 4);
  uint64_t* ext = malloc(sizeof(uint64_t) * ((meta_off + 2) / 1 + 2));
  uint32_t nb = 0;
  for (uint64_t q = meta_off; q < bloom_off - 4; nb++) {
    ext[nb] = be32(file + q);
    q += 6 + ((uint64_t)file[q + 4] << 8 | file[q + 5]);
  }
  ext[nb] = meta_off;
  tpz_ctx* ctx = NULL;
  CHECK_TPZ(tpz_ctx_create(0, &ctx));
  uint64_t bound = 0;
  CHECK_TPZ(tpz_host_decoded_bound(file, ext, nb, &bound));
  tpz_host_columns o;
  memset(&o, 0, sizeof o);
  o.data_cap = tpz_data_capacity(bound, nb);
  o.h_data = malloc(o.data_cap);
  o.ends_cap = 2 * (bound / 4 + 16);
  o.h_ends = malloc(o.ends_cap * 4);
  o.h_first = malloc((nb + 1) * 8);
  o.h_count = malloc(nb * 4);
  o.h_status = malloc(nb);
  o.h_crc = malloc(nb * 4);
  o.h_spill_off = malloc(nb * 8);
  uint64_t spill_used = 0;
  o.h_spill_used = &spill_used;
  o.h_dext = malloc((nb + 1) * 8);
  CHECK_TPZ(tpz_decode_blocks_host(ctx, file, ext, nb, &o, chunk));
  uint64_t ents = 0;
  for (uint32_t b = 0; b < nb; b++) {
    if (o.h_status[b] != TPZ_BLOCK_OK) {
      printf("block %u: status %u\n", b, o.h_status[b]);
      return 1;
    }
    const uint64_t s = tpz_slot_base(o.h_dext[b], b);
    const uint32_t n = (uint32_t)(o.h_first[b + 1] - o.h_first[b]);
    const uint32_t* en = o.h_ends + 2 * o.h_first[b];
    const uint64_t vs = tpz_value_start(n ? en[2 * (n - 1)] : 0);
    for (uint32_t j = 0; j < n; j++, ents++) {
      const uint32_t k0 = j ? en[2 * (j - 1)] : 0, v0 = j ? en[2 * (j - 1) + 1] : 0;
      hex(o.h_data + s + k0, en[2 * j] - k0);
      putchar(' ');
      hex(o.h_data + s + vs + v0, en[2 * j + 1] - v0);
      putchar('\n');
    }
  }
  printf("ok sst %u %llu\n", nb, (unsigned long long)ents);
  tpz_ctx_destroy(ctx);
  return 0;
}

static void* host_alloc(size_t n, int pinned) {
  void* p = NULL;
  if (pinned) {
    if (hipHostMalloc(&p, n ? n : 1, hipHostMallocDefault) != hipSuccess) return NULL;
    return p;
  }
  return malloc(n ? n : 1);
}

int main(int argc, char** argv) {
  if (argc > 2 && strcmp(argv[1], "--sst") == 0)
    return sst_mode(argv[2], argc > 3 ? (uint32_t)strtoul(argv[3], NULL, 10) : 0);
  const uint64_t n_entries = argc > 1 ? strtoull(argv[1], NULL, 10) : 20000;
  const uint32_t chunk = argc > 2 ? (uint32_t)strtoul(argv[2], NULL, 10) : 37;
  const int pinned = argc > 3 ? atoi(argv[3]) : 0;
  const int codec = argc > 4 ? atoi(argv[4]) : 0;
  uint64_t seed = 0x5EEDC0DEull;
  uint64_t* kpos = malloc((n_entries + 1) * sizeof(uint64_t));
  uint64_t* vpos = malloc((n_entries + 1) * sizeof(uint64_t));
  uint8_t* keys = malloc(16 * n_entries + 1);
  uint8_t* vals = malloc(200 * n_entries + 1);
  kpos[0] = vpos[0] = 0;
  for (uint64_t e = 0; e < n_entries; e++) {
    for (int i = 0; i < 8; i++) keys[16 * e + i] = (uint8_t)(e >> (56 - 8 * i));
    const uint64_t r = splitmix(&seed);
    memcpy(keys + 16 * e + 8, &r, 8);
    kpos[e + 1] = 16 * (e + 1);
    const uint64_t vl = splitmix(&seed) % 200;
    for (uint64_t i = 0; i < vl; i++) vals[vpos[e] + i] = (uint8_t)splitmix(&seed);
    vpos[e + 1] = vpos[e] + vl;
  }
  const uint64_t cap = 2 * (kpos[n_entries] + vpos[n_entries]) + 8192;
  uint8_t* blocks = host_alloc(cap, pinned);
  uint64_t* ext = malloc((n_entries + 3) * sizeof(uint64_t));
  uint64_t nb = 0, len = 0;
  CHECK_TPZ(tpz_build_blocks(keys, kpos, vals, vpos, n_entries, 4096, blocks, cap, ext,
                             n_entries + 3, &nb, &len));
  const uint64_t bad = nb / 2;                      /* a corrupted payload byte: CRC mismatch */
  blocks[ext[bad] + 7] ^= 0x40;
  /* the blocks as the decode receives them: compressed (codec 2 / 3) or as built */
  uint8_t* in = blocks;
  uint64_t* iext = ext;
  uint64_t ilen = len;
  if (codec == 2 || codec == 3) {
    const uint64_t ccap = 32 * nb + 2 * len + 8192;
    in = host_alloc(ccap, pinned);
    iext = malloc((nb + 3) * sizeof(uint64_t));
    if (codec == 2)
      CHECK_TPZ(tpz_snappy_encode_blocks(blocks, ext, nb, in, ccap, iext, &ilen));
    else
      CHECK_TPZ(tpz_lz4_encode_blocks(blocks, ext, nb, in, ccap, iext, &ilen));
  }
  /* a stream the codec rejects (codec 2: a literal longer than the input; codec 3: a size
   * prefix with no stream): Err in the reference, CODEC_ERROR here */
  const uint64_t broken = nb;
  if (codec == 2 || codec == 3) {
    static const uint8_t snap_bad[] = {0x05, 0x10, 'a', 'b', 2};
    static const uint8_t lz4_bad[] = {5, 0, 0, 0, 0x50, 'h', 3};
    const uint8_t* bb = codec == 2 ? snap_bad : lz4_bad;
    const size_t bl = codec == 2 ? sizeof snap_bad : sizeof lz4_bad;
    memcpy(in + ilen, bb, bl);
    ilen += bl;
    iext[nb + 1] = ilen;
    nb += 1;
  }
  /* the spilled block: n = 64, every offset 0, one entry (2000-byte key, value "abc") */
  const uint32_t nrep = 64, kl = 2000;
  uint8_t* p = in + ilen;
  size_t q = 0;
  p[q++] = 0;
  p[q++] = (uint8_t)nrep;
  for (uint32_t i = 0; i < nrep; i++) p[q++] = 0, p[q++] = 0;
  p[q++] = (uint8_t)(kl >> 8);
  p[q++] = (uint8_t)kl;
  for (uint32_t i = 0; i < kl; i++) p[q++] = (uint8_t)('A' + i % 26);
  p[q++] = 0;
  p[q++] = 3;
  memcpy(p + q, "abc", 3);
  q += 3;
  const uint32_t pc = tpz_host_crc32(p, q);
  p[q++] = (uint8_t)(pc >> 24), p[q++] = (uint8_t)(pc >> 16), p[q++] = (uint8_t)(pc >> 8),
  p[q++] = (uint8_t)pc;
  p[q++] = 1;
  iext[nb + 1] = ilen + q;
  nb += 1;
  ilen += q;

  tpz_ctx* ctx = NULL;
  CHECK_TPZ(tpz_ctx_create(0, &ctx));
  tpz_host_columns o;
  memset(&o, 0, sizeof o);
  uint64_t bound = 0;
  CHECK_TPZ(tpz_host_decoded_bound(in, iext, (uint32_t)nb, &bound));
  o.data_cap = tpz_data_capacity(bound, nb);
  o.h_data = host_alloc(o.data_cap, pinned);
  o.h_dext = malloc((nb + 1) * sizeof(uint64_t));
  o.ends_cap = 2 * (n_entries + nrep);
  o.h_ends = host_alloc(o.ends_cap * sizeof(uint32_t), pinned);
  o.h_first = malloc((nb + 1) * sizeof(uint64_t));
  o.h_count = malloc(nb * sizeof(uint32_t));
  o.h_status = malloc(nb);
  o.h_crc = malloc(nb * sizeof(uint32_t));
  o.spill_cap = 1 << 20;
  o.h_spill = host_alloc(o.spill_cap, pinned);
  o.h_spill_off = malloc(nb * sizeof(uint64_t));
  uint64_t spill_used = 0;
  o.h_spill_used = &spill_used;
  if (!blocks || !o.h_data || !o.h_ends || !o.h_spill) return 1;

  CHECK_TPZ(tpz_decode_blocks_host(ctx, in, iext, (uint32_t)nb, &o, chunk)); /* warm */
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  CHECK_TPZ(tpz_decode_blocks_host(ctx, in, iext, (uint32_t)nb, &o, chunk));
  clock_gettime(CLOCK_MONOTONIC, &t1);
  const double dt = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);

  const uint64_t nbuilt = (codec == 2 || codec == 3) ? nb - 2 : nb - 1;
  if (nbuilt != nb - 1) {
    if (o.h_status[broken] != TPZ_BLOCK_CODEC_ERROR || o.h_count[broken] != 0 ||
        o.h_first[broken + 1] != o.h_first[broken]) {
      printf("broken codec block: status %u\n", o.h_status[broken]);
      return 1;
    }
  }
  uint64_t e = 0;
  for (uint64_t b = 0; b < nbuilt; b++) {
    const uint32_t want_crc = tpz_host_crc32(blocks + ext[b], ext[b + 1] - ext[b] - 5);
    if (o.h_dext[b + 1] - o.h_dext[b] != ext[b + 1] - ext[b]) {
      printf("block %llu: decoded length %llu, built %llu\n", (unsigned long long)b,
             (unsigned long long)(o.h_dext[b + 1] - o.h_dext[b]),
             (unsigned long long)(ext[b + 1] - ext[b]));
      return 1;
    }
    const uint32_t n = (uint32_t)(o.h_first[b + 1] - o.h_first[b]);
    if (b == bad) {
      /* reference: Err("checksum: expected E, actual A"); entries are still generated */
      if (o.h_status[b] != TPZ_BLOCK_CHECKSUM_MISMATCH || o.h_crc[b] != want_crc || n != 0) {
        printf("block %llu: status %u crc %08x want %08x\n", (unsigned long long)b, o.h_status[b],
               o.h_crc[b], want_crc);
        return 1;
      }
      const uint8_t* pl = blocks + ext[b];
      e += (uint64_t)(pl[0] << 8 | pl[1]);           /* n is intact: byte 7 is an offset */
      continue;
    }
    if (o.h_status[b] != TPZ_BLOCK_OK || o.h_crc[b] != want_crc || n != o.h_count[b]) {
      printf("block %llu: status %u crc %08x want %08x\n", (unsigned long long)b, o.h_status[b],
             o.h_crc[b], want_crc);
      return 1;
    }
    const uint64_t s = tpz_slot_base(o.h_dext[b], b);
    const uint32_t* en = o.h_ends + 2 * o.h_first[b];
    const uint64_t K = n ? en[2 * (n - 1)] : 0, vs = tpz_value_start(K);
    for (uint32_t j = 0; j < n; j++, e++) {
      const uint32_t k0 = j ? en[2 * (j - 1)] : 0, k1 = en[2 * j];
      const uint32_t v0 = j ? en[2 * (j - 1) + 1] : 0, v1 = en[2 * j + 1];
      if (e >= n_entries || k1 - k0 != kpos[e + 1] - kpos[e] ||
          memcmp(o.h_data + s + k0, keys + kpos[e], k1 - k0) != 0 ||
          v1 - v0 != vpos[e + 1] - vpos[e] ||
          memcmp(o.h_data + s + vs + v0, vals + vpos[e], v1 - v0) != 0) {
        printf("block %llu entry %u differs\n", (unsigned long long)b, j);
        return 1;
      }
    }
  }
  if (e != n_entries) {
    printf("%llu of %llu entries accounted for\n", (unsigned long long)e,
           (unsigned long long)n_entries);
    return 1;
  }
  /* the spilled block: 64 copies of the one entry, from its record */
  const uint64_t sb = nb - 1;
  if (o.h_status[sb] != TPZ_BLOCK_OK_SPILLED || o.h_count[sb] != nrep ||
      o.h_first[sb + 1] - o.h_first[sb] != nrep) {
    printf("spilled block: status %u count %u\n", o.h_status[sb], o.h_count[sb]);
    return 1;
  }
  const uint8_t* rec = o.h_spill + o.h_spill_off[sb];
  const uint32_t* re = (const uint32_t*)rec;
  const uint8_t* rs = rec + tpz_layout_spill_stream(nrep);
  const uint64_t rvs = tpz_value_start((uint64_t)nrep * kl);
  for (uint32_t j = 0; j < nrep; j++) {
    const uint32_t* dj = o.h_ends + 2 * (o.h_first[sb] + j);
    if (re[2 * j] != (j + 1) * kl || re[2 * j + 1] != (j + 1) * 3 || dj[0] != re[2 * j] ||
        dj[1] != re[2 * j + 1] || memcmp(rs + j * kl, p + 2 + 2 * nrep + 2, kl) != 0 ||
        memcmp(rs + rvs + 3 * j, "abc", 3) != 0) {
      printf("spilled entry %u differs\n", j);
      return 1;
    }
  }
  printf("ok %llu %llu %.2f\n", (unsigned long long)nb, (unsigned long long)e,
         (double)ilen / dt / (double)(1ull << 30));
  tpz_ctx_destroy(ctx);
  return 0;
}
