// tpz_crc.hip — gfx950 kernels for CRC-32 over long byte ranges in HBM.
//
// Restates, on the device, for a batch of ranges (whole SST file images, or any buffers):
//   checksum::calculate_checksum (crc32fast)      src/checksum.rs:6-10
//   FileObject::open's whole-file verification    src/table/file_object.rs:57-78
//     (crc over buf[..size-4], compared with the big-endian u32 in buf[size-4..])
//
// All arithmetic is on raw CRCs (init 0, no xorout): R0(M). For the standard CRC,
//   crc32(M) = ~(R0(M) ^ Z_|M|(0xFFFFFFFF)),  Z_n(a) = the register after n zero bytes from a,
// and R0 is linear: R0(A || B) = Z_|B|(R0(A)) ^ R0(B); leading zero bytes leave R0 unchanged.
//
// Work split: the buffer is cut into absolute 8 KiB windows (addresses taken
// from d_src rounded down to 16 B). Every wave owns a contiguous span of windows. For each
// (window, range) overlap it computes R0 of the overlap's "main" part (the range up to its last
// 16-byte boundary): lane l folds the 128-byte run that ends 128*l bytes before the overlap's end
// (8 aligned dwordx4 loads straight into registers, bytes before the range masked to zero) with
// slice-by-4 lookups, shifts it by 128*l with the shift-by-16*2^j operators (bits of l), and the
// wave XORs the lanes. While a window is folded, the next one's loads are in flight when the same
// range covers it. The wave folds the parts of one range in order (Horner: acc = Z_d(acc) ^ part,
// d = the distance between the two parts' ends, one window for whole windows), and when it leaves
// the range shifts acc to the end of the range's main part and XORs it into the range's
// accumulator (atomicXor, order-free: one atomic per wave and range). The current range's
// geometry stays in registers, so whole windows of one range load no extents. A per-range finish
// kernel applies the init term, the (< 16) tail bytes, the xorout and, for files, the trailer
// compare.
//
// The hot lookups are conflict-free: the slice-by-4 tables sit in LDS replicated 32 times, word
// ((t*256 + b)*32 + r) = T_t[b], and lane l reads replica l % 32, so a ds_read_b32 of 32 lanes
// hits 32 distinct banks whatever the data (128 KiB). The lane-shift operators (24 KiB) are in LDS
// too; the rare window shifts and the finish kernel read the global tables.
//
// Global tables (built by tpz_api.cpp, (16 + 4 * kRangeShiftOps) x 256 u32):
//   0..15           T_0..T_15, T_k[b] = R0(b || 0^k)
//   16 + 4j + i     T_{n-1-i} for n = 16 * 2^j, j = 0..kRangeShiftOps-1   (Z_n operator)
// Replicated table (128 KiB): rep[(t*256 + b)*32 + r] = T_t[b], t = 0..3, r = 0..31.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tpz_internal.h"

namespace tpz {

namespace {

typedef uint32_t u32;
typedef uint64_t u64;

constexpr int kWave = 64;
constexpr int kWaves = 16;
constexpr int kThreads = kWave * kWaves;
#ifndef TPZ_CRC_RUN_LOG
#define TPZ_CRC_RUN_LOG 7                          // diagnostic builds vary the lane run
#endif
constexpr u32 kLaneRun = 1u << TPZ_CRC_RUN_LOG;    // bytes folded per lane per window (128)
constexpr int kWinLog = TPZ_CRC_RUN_LOG + 6;
constexpr u64 kWin = 1ull << kWinLog;              // 8 KiB = 64 lanes x 128 B
static_assert(kWin == (u64)kLaneRun * kWave, "window");
constexpr int kJLane = TPZ_CRC_RUN_LOG - 4;        // lane l shifts by 128*l: operators j = 3..8
constexpr int kLaneOps = 6;
constexpr int kJWin = kWinLog - 4;                 // the shift-by-one-window operator
constexpr int kRepWords = kCrcRepWords;            // 4 x 256 x 32
constexpr int kLdsWords = kRepWords + (kLaneOps + 1) * 4 * 256;  // + the window op
static_assert(kLdsWords * 4 <= 163840, "LDS");

__device__ __forceinline__ u32 lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
__device__ __forceinline__ u32 uni(u32 x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ u64 uni64(u64 x) {
  const u32 lo = __builtin_amdgcn_readfirstlane((u32)x);
  const u32 hi = __builtin_amdgcn_readfirstlane((u32)(x >> 32));
  return ((u64)hi << 32) | lo;
}
__device__ __forceinline__ u32 xor3(u32 a, u32 b, u32 c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Z_n for n = 16 * 2^j from four byte tables at `t` (T_{n-1}, T_{n-2}, T_{n-3}, T_{n-4}).
__device__ __forceinline__ u32 zop(const u32* t, u32 a) {
  return xor3(t[a & 0xFF], t[256 + ((a >> 8) & 0xFF)], t[512 + ((a >> 16) & 0xFF)]) ^
         t[768 + (a >> 24)];
}
__device__ __forceinline__ const u32* gop(const u32* g, int j) { return g + (16 + 4 * j) * 256; }

// One slice-by-4 step: x = register ^ next message word; returns the register after the word.
__device__ __forceinline__ u32 slice4(const u32* rep, u32 r, u32 x) {
  const u32 a0 = rep[((3u * 256u + (x & 0xFF)) << 5) + r];
  const u32 a1 = rep[((2u * 256u + ((x >> 8) & 0xFF)) << 5) + r];
  const u32 a2 = rep[((1u * 256u + ((x >> 16) & 0xFF)) << 5) + r];
  const u32 a3 = rep[((x >> 24) << 5) + r];
  return xor3(a0, a1, a2) ^ a3;
}

// Zero the bytes of a 16-byte chunk whose offset within the chunk is < k (k in 0..16).
__device__ __forceinline__ uint4 zero_below(uint4 v, u32 k) {
  const u64 lo = (u64)v.y << 32 | v.x, hi = (u64)v.w << 32 | v.z;
  const u64 mlo = k >= 8 ? 0ull : (~0ull << (8 * k));
  const u64 mhi = k >= 16 ? 0ull : (k <= 8 ? ~0ull : (~0ull << (8 * (k - 8))));
  const u64 a = lo & mlo, b = hi & mhi;
  return make_uint4((u32)a, (u32)(a >> 32), (u32)b, (u32)(b >> 32));
}

// Geometry of range r in the aligned address space X = offset + delta (delta = d_src & 15):
// CRC region [s, e), main part [s, A) with A = max(s, e & ~15) (16-aligned when non-empty),
// tail [A, e) (< 16 bytes). `valid` is false when the range is shorter than the trailer.
struct RangeGeo {
  u64 s, e, A;
  bool valid;
};
__device__ __forceinline__ RangeGeo range_geo(u64 lo, u64 hi, u32 delta, u32 trailer) {
  RangeGeo g;
  g.valid = hi >= lo + trailer;
  g.s = lo + delta;
  g.e = g.valid ? hi - trailer + delta : g.s;
  const u64 ea = g.e & ~15ull;
  g.A = ea > g.s ? ea : g.s;
  return g;
}

struct CrcParams {
  const uint8_t* base;  // d_src rounded down to 16 bytes
  const u64* ext;
  u32 n_ranges;
  u32 delta;            // d_src - base
  u32 trailer;          // 0: plain CRC; 4: FileObject trailer (BE u32 after the CRC region)
  u64 n_windows;        // windows of the aligned space covering [0, src_bytes + delta)
  const u32* tables;    // global tables (ids above)
  const u32* rep;       // replicated slice-by-4 tables
  u32* acc;             // per range: R0 of the main part (XOR of the waves' shifted folds)
  u32* crc;             // out
  uint8_t* status;      // out (verify mode) or null
};

// Z_n(a) for any n < 16 * 2^kRangeShiftOps: the n mod 16 bytes with the slice tables, then the
// shift-by-16*2^j operators for the bits of n / 16.
__device__ __forceinline__ u32 zshift_any(const u32* g, u32 a, u64 n) {
  const u32 k = (u32)(n & 15);
  if (k) {
    u32 r = k >= 4 ? 0u : (a >> (8 * k));
    for (u32 i = 0; i < 4 && i < k; i++) r ^= g[(k - 1 - i) * 256 + ((a >> (8 * i)) & 0xFF)];
    a = r;
  }
  u64 m = n >> 4;
  for (int j = 0; m; j++, m >>= 1)
    if (m & 1) a = zop(gop(g, j), a);
  return a;
}

// ------------------------------------------------------------------ window kernel
__global__ __launch_bounds__(kThreads, 1) void crc_window_kernel(CrcParams p) {
  __shared__ __attribute__((aligned(16))) u32 lds[kLdsWords];
  const u32* rep = lds;
  const u32* lop = lds + kRepWords;                 // lane-shift operator k at lop + 1024 k
  const u32* wop = lop + 1024 * kLaneOps;           // shift by one window
  const u32 lane = lane_id();
  const u32 rl = lane & 31u;
  const u64 nw = (u64)gridDim.x * kWaves;
  const u64 wave = (u64)blockIdx.x * kWaves + uni(threadIdx.x >> 6);
  const u64 per = (p.n_windows + nw - 1) / nw;
  const u64 g0 = wave * per;
  const u64 g1 = min(p.n_windows, g0 + per);
  const bool live = g0 < g1 && p.n_ranges != 0;

  // The span's first range and first window are found and that window's loads issued before the
  // tables are staged in LDS, so its HBM latency overlaps the staging (every workgroup stages
  // 156 KiB at the start)
  u32 r = 0;
  u32 cur = ~0u, acc = 0;   // the range being folded, R0 of its parts so far ending at `last`
  u64 last = 0, cur_A = 0;
  // the next window's runs, loaded while the current one is folded when the range covers it
  constexpr int kC = (int)(kLaneRun / 16);
  uint4 pf[kC];
  u64 pf_g = ~0ull;
  u32 pf_r = ~0u;
  // range r's geometry and end stay in registers: consecutive windows of one range (the common
  // case, files are MiBs) need no extent loads; range r + 1 starts where r ends
  u64 hiX = 0;
  RangeGeo Gr = range_geo(0, 0, 0, 0);
  if (live) {
    // first range whose end (aligned space) lies beyond the span's start (ext is non-decreasing)
    const u64 t = g0 << kWinLog;
    u32 lo = 0, hi = p.n_ranges;  // smallest r with ext[r+1] + delta > t
    while (lo < hi) {
      const u32 mid = (lo + hi) >> 1;
      if (uni64(p.ext[mid + 1]) + p.delta > t) hi = mid; else lo = mid + 1;
    }
    r = lo;
    if (r < p.n_ranges) {
      hiX = uni64(p.ext[r + 1]) + p.delta;
      Gr = range_geo(uni64(p.ext[r]), hiX - p.delta, p.delta, p.trailer);
      if (Gr.valid && t >= Gr.s && t + kWin <= Gr.A) {   // the first window lies inside range r
        const uint8_t* x = p.base + t + kWin - (u64)kLaneRun * (lane + 1);
#pragma unroll
        for (int c = 0; c < kC; c++) pf[c] = *reinterpret_cast<const uint4*>(x + 16 * c);
        pf_g = g0;
        pf_r = r;
      }
    }
  }
  {
    const uint4* g = reinterpret_cast<const uint4*>(p.rep);
    const uint4* o = reinterpret_cast<const uint4*>(gop(p.tables, kJLane));
    const uint4* w = reinterpret_cast<const uint4*>(gop(p.tables, kJWin));
    uint4* d = reinterpret_cast<uint4*>(lds);
    constexpr int kRep4 = kRepWords / 4, kOps4 = kLaneOps * 256;
    for (int i = threadIdx.x; i < kLdsWords / 4; i += kThreads)
      d[i] = i < kRep4 ? g[i] : (i < kRep4 + kOps4 ? o[i - kRep4] : w[i - kRep4 - kOps4]);
    __syncthreads();
  }
  if (!live) return;
  for (u64 g = g0; g < g1 && r < p.n_ranges; g++) {
    const u64 w0 = g << kWinLog, w1 = w0 + kWin;
    while (hiX <= w0 && r + 1 < p.n_ranges) {
      r++;
      const u64 lo = hiX - p.delta;
      hiX = uni64(p.ext[r + 1]) + p.delta;
      Gr = range_geo(lo, hiX - p.delta, p.delta, p.trailer);
    }
    if (hiX <= w0) break;
    u32 rr = r;
    RangeGeo G = Gr;
    u64 rhi = hiX;
    for (;;) {
      const u64 a = max(w0, G.s), b = min(w1, G.A);
      if (G.valid && a < b) {
        // lane l: the run ending kLaneRun*l bytes before b (b is 16-aligned); chunks wholly
        // before the range are not loaded (their address may lie before the buffer) and read as 0
        const int64_t run0 = (int64_t)b - (int64_t)kLaneRun * (int64_t)(lane + 1);
        uint4 v[kC];
        if (pf_g == g && pf_r == rr && a == w0 && b == w1) {
#pragma unroll
          for (int c = 0; c < kC; c++) v[c] = pf[c];
        } else {
#pragma unroll
          for (int c = 0; c < kC; c++) {
            const int64_t x = run0 + 16 * c;
            v[c] = make_uint4(0, 0, 0, 0);
            if (x + 16 > (int64_t)a) {
              v[c] = *reinterpret_cast<const uint4*>(p.base + x);
              if (x < (int64_t)a) v[c] = zero_below(v[c], (u32)((int64_t)a - x));
            }
          }
        }
        if (g + 1 < g1 && G.A >= w1 + kWin) {       // the range covers the next window: load it
          const uint8_t* nx = p.base + w1 + kWin - (u64)kLaneRun * (lane + 1);
#pragma unroll
          for (int c = 0; c < kC; c++) pf[c] = *reinterpret_cast<const uint4*>(nx + 16 * c);
          pf_g = g + 1;
          pf_r = rr;
        }
        u32 R = 0;
#pragma unroll
        for (int c = 0; c < kC; c++) {
          R = slice4(rep, rl, R ^ v[c].x);
          R = slice4(rep, rl, R ^ v[c].y);
          R = slice4(rep, rl, R ^ v[c].z);
          R = slice4(rep, rl, R ^ v[c].w);
        }
        // lane l sits kLaneRun*l bytes before b: Z_{run*l} = product of Z_{run*2^k} for bits k of l
#pragma unroll
        for (int k = 0; k < kLaneOps; k++)
          if (lane & (1u << k)) R = zop(lop + 1024 * k, R);
        for (int o = 32; o >= 1; o >>= 1) R ^= __shfl_xor(R, o);
        R = uni(R);
        if (rr == cur) {
          // the previous part ended at `last` = w0; this one ends at b
          acc = (b - last == kWin ? zop(wop, acc) : zshift_any(p.tables, acc, b - last)) ^ R;
        } else {
          if (cur != ~0u && lane == 0)
            atomicXor(p.acc + cur, zshift_any(p.tables, acc, cur_A - last));
          cur = rr;
          cur_A = G.A;
          acc = R;
        }
        last = b;
      }
      // the next range starts at this one's end: in this window only if that is before w1
      if (rhi >= w1 || rr + 1 >= p.n_ranges) break;
      rr++;
      const u64 lo = rhi - p.delta;
      rhi = uni64(p.ext[rr + 1]) + p.delta;
      G = range_geo(lo, rhi - p.delta, p.delta, p.trailer);
    }
  }
  if (cur != ~0u && lane == 0) atomicXor(p.acc + cur, zshift_any(p.tables, acc, cur_A - last));
}

// ------------------------------------------------------------------ finish kernel
__global__ __launch_bounds__(256) void crc_finish_kernel(CrcParams p) {
  const u32 r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= p.n_ranges) return;
  const RangeGeo G = range_geo(p.ext[r], p.ext[r + 1], p.delta, p.trailer);
  if (!G.valid) {                      // file_object.rs:69: buf[size - CHECKSUM_SIZE..] panics
    p.crc[r] = 0;
    if (p.status) p.status[r] = TPZ_BLOCK_MALFORMED;
    return;
  }
  u32 R = p.acc[r];                    // R0 of the main part [s, A)
  R ^= zshift_any(p.tables, 0xFFFFFFFFu, G.A - G.s);  // init 0xFFFFFFFF ahead of the main part
  for (u64 x = G.A; x < G.e; x++) R = (R >> 8) ^ p.tables[(R ^ p.base[x]) & 0xFF];
  const u32 crc = ~R;
  p.crc[r] = crc;
  if (p.status) {
    const uint8_t* t = p.base + G.e;   // the trailer: big-endian u32 (file_object.rs:69)
    const u32 stored = ((u32)t[0] << 24) | ((u32)t[1] << 16) | ((u32)t[2] << 8) | t[3];
    p.status[r] = crc == stored ? TPZ_BLOCK_OK : TPZ_BLOCK_CHECKSUM_MISMATCH;  // checksum.rs:17
  }
}

}  // namespace

void launch_crc_ranges(const CrcLaunch& a, hipStream_t stream) {
  CrcParams p;
  const uintptr_t sp = reinterpret_cast<uintptr_t>(a.src);
  p.delta = (u32)(sp & 15u);
  p.base = a.src - p.delta;
  p.ext = a.ext;
  p.n_ranges = a.n_ranges;
  p.trailer = a.trailer;
  p.n_windows = (a.src_bytes + p.delta + kWin - 1) >> kWinLog;
  p.tables = a.tables;
  p.rep = a.rep;
  p.acc = a.acc;
  p.crc = a.crc;
  p.status = a.status;
  // enough waves for the windows, at most one 16-wave workgroup per CU
  u64 wgs = (p.n_windows + kWaves - 1) / kWaves;
  if (wgs > a.num_cus) wgs = a.num_cus;
  if (wgs == 0) wgs = 1;
  hipLaunchKernelGGL(crc_window_kernel, dim3((u32)wgs), dim3(kThreads), 0, stream, p);
  if (!a.acc_only)
    hipLaunchKernelGGL(crc_finish_kernel, dim3((a.n_ranges + 255) / 256), dim3(256), 0, stream, p);
}

}  // namespace tpz

// ------------------------------------------------------------------ copy probe (diagnostic)
// The box's HBM copy rate for bench.py's roofline.copy_ceiling: one 16-byte piece per thread and
// a grid covering the buffer (each wave loads, stores and ends; MI355X_MICROARCH.md's 6.3 TB/s
// float4 copy). Persistent or grid-stride copies wait on their own store acknowledgements (the
// next load's vmcnt counts the stores issued before it) and run at 4.3-4.8 TB/s
// (tools/ubench_bw.hip), so they understate the ceiling.
namespace {
__global__ __launch_bounds__(256) void copy_probe_kernel(const uint4* __restrict__ s, uint4* __restrict__ d,
                                                         unsigned long long n16) {
  const unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x;
  if (i < n16) d[i] = s[i];
}
}  // namespace
extern "C" int tpz_debug_copy(void* dst, const void* src, unsigned long long bytes, void* stream) {
  const unsigned long long n16 = bytes / 16;
  if (!n16) return 0;
  if ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15u) return -1;
  const unsigned long long grid = (n16 + 255) / 256;
  if (grid > 0x7FFFFFFFull) return -1;
  hipLaunchKernelGGL(copy_probe_kernel, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const uint4*>(src), reinterpret_cast<uint4*>(dst), n16);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
