// Diagnostic (not shipped): HBM write-pattern microbenchmark for the decode output layout.
// Each wave handles blocks b = wave, wave + nwaves, ... and, like the decoder, reads a 4155-B
// block and writes 4 column pieces (keys 544 B, values 3400 B, kend 136 B, vend 136 B) with
// 16-B lane-coalesced stores. Patterns differ only in WHERE the pieces go.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef uint32_t u32;
typedef uint64_t u64;
constexpr u32 NB = 1u << 20, BL = 4155, KB = 544, VB = 3400, EB = 136;

template <bool NT = false>
__device__ inline void put(uint8_t* dst, u32 bytes, u32 lane, u32 v, bool pad128) {
  u32 nb = pad128 ? ((bytes + 127) & ~127u) : bytes;
  for (u32 c = lane; c * 16 < nb; c += 64) {
    typedef u32 u32x4 __attribute__((ext_vector_type(4)));
    u32x4 val = {v, c, 0, 0};
    if (NT) __builtin_nontemporal_store(val, reinterpret_cast<u32x4*>(dst + c * 16));
    else *reinterpret_cast<u32x4*>(dst + c * 16) = val;
  }
}

// MODE 3: 128-B padded slots, but values written entry-owned: lane i (34 entries of 100 B)
// writes the 16-B chunks starting inside its entry, so one store instruction scatters 64 lanes
// ~100 B apart (7 instructions fill 3400 B) instead of 1 KiB contiguous.
__device__ inline void put_scatter(uint8_t* dst, u32 lane, u32 v) {
  if (lane < 34) {
    u32 f = (lane * 100 + 15) / 16, g = (lane * 100 + 100 + 15) / 16;
    for (u32 c = f; c < g; c++) *reinterpret_cast<uint4*>(dst + c * 16) = make_uint4(v, c, 0, 0);
  }
  if (lane < 3) *reinterpret_cast<uint4*>(dst + (213 + lane) * 16) = make_uint4(v, lane, 0, 0);
}

template <int MODE, bool READ>
__global__ __launch_bounds__(1024) void k(const uint8_t* src, uint8_t* keys, uint8_t* vals, uint8_t* ke, uint8_t* ve) {
  const u32 lane = threadIdx.x & 63;
  const u32 wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 nw = gridDim.x * 16;
  u32 acc = 0;
  for (u32 b = blockIdx.x * 16 + wid; b < NB; b += nw) {
    if (READ) {
      const uint8_t* s = src + (u64)b * BL;
      for (u32 o = lane * 16; o < BL - 16; o += 1024) {
        const uint4* q = reinterpret_cast<const uint4*>(((u64)(s + o)) & ~15ull);
        if (MODE == 5) acc += __builtin_nontemporal_load(&q->x);
        else acc += q->x;
      }
    }
    u64 kb, vb, eb;
    if (MODE == 0) {  // slotted, 64-B aligned (first layout): 64-B aligned per-block regions, sparse
      kb = ((((u64)b * BL) + 63) & ~63ull) + 128ull * b; vb = kb;
      eb = 16ull * (((u64)b * BL) / 96 + b) * 4;
    } else if (MODE == 1 || MODE == 3 || MODE == 4 || MODE == 5) {  // slotted, 128-B aligned, whole 128-B lines
      kb = ((((u64)b * BL) + 127) & ~127ull) + 256ull * b; vb = kb;
      eb = (((u64)b * 256));
    } else {  // dense: per-block regions packed back to back (16-B rounded)
      kb = (u64)b * KB; vb = (u64)b * VB; eb = (u64)b * 144;
    }
    if (MODE >= 4) {  // 4: 128-B slots with nontemporal stores; 5: + nontemporal loads
      put<true>(keys + kb, KB, lane, acc, true);
      put<true>(vals + vb, VB, lane, acc, true);
      put<true>(ke + eb, EB, lane, acc, true);
      put<true>(ve + eb, EB, lane, acc, true);
    } else {
      put(keys + kb, KB, lane, acc, MODE == 1 || MODE == 3);
      if (MODE == 3) put_scatter(vals + vb, lane, acc); else put(vals + vb, VB, lane, acc, MODE == 1);
      put(ke + eb, EB, lane, acc, MODE == 1);
      put(ve + eb, EB, lane, acc, MODE == 1);
    }
  }
}

template <int M, bool R> float run(uint8_t* s, uint8_t* a, uint8_t* b, uint8_t* c, uint8_t* d) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  k<M, R><<<256, 1024>>>(s, a, b, c, d);
  (void)hipDeviceSynchronize();
  float best = 1e9;
  for (int i = 0; i < 5; i++) {
    (void)hipEventRecord(e0);
    k<M, R><<<256, 1024>>>(s, a, b, c, d);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  return best;
}

int main() {
  uint8_t *s, *a, *b, *c, *d;
  size_t cap = (size_t)NB * (BL + 512) + (1 << 20);
  (void)hipMalloc(&s, (size_t)NB * BL + 4096);
  (void)hipMalloc(&a, cap); (void)hipMalloc(&b, cap); (void)hipMalloc(&c, cap); (void)hipMalloc(&d, cap);
  const char* names[] = {"slotted-64B", "slotted-128B padded", "dense", "128B, scattered values",
                         "128B padded, nt stores", "128B, nt stores+loads"};
  float w[6] = {run<0, false>(s, a, b, c, d), run<1, false>(s, a, b, c, d), run<2, false>(s, a, b, c, d),
                run<3, false>(s, a, b, c, d), run<4, false>(s, a, b, c, d), run<5, false>(s, a, b, c, d)};
  float rw[6] = {run<0, true>(s, a, b, c, d), run<1, true>(s, a, b, c, d), run<2, true>(s, a, b, c, d),
                 run<3, true>(s, a, b, c, d), run<4, true>(s, a, b, c, d), run<5, true>(s, a, b, c, d)};
  double wb = (double)NB * (KB + VB + 2 * EB), rb = (double)NB * BL;
  for (int m = 0; m < 6; m++)
    printf("%-24s write-only %.3f ms (%.0f GB/s)   read+write %.3f ms (%.0f GB/s)\n", names[m], w[m],
           wb / w[m] / 1e6, rw[m], (wb + rb) / rw[m] / 1e6);
  return 0;
}
