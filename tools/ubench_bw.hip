// Diagnostic (not shipped): HBM bandwidth ceilings on this MI355X for the traffic mix of the
// decode (read N bytes, write ~N bytes, 4.36 GB each way) — what any kernel of this shape can
// reach. Variants:
//   read            sum-reduce of N bytes (16-B loads, 4 in flight per lane)
//   write           fill of N bytes (16-B stores)
//   copy[_ilpK]     N bytes -> N bytes, K 16-B loads in flight per lane (grid = 8 x CUs x 256)
//   copy_nt         the same with nontemporal stores
//   copy_ntl        nontemporal loads and stores
//   copy_gG         copy with G x CUs workgroups of 256 threads
//   copy_wave4k     persistent, one wave per 4 KiB chunk, 1 KiB per wave instruction
//   memcpy          hipMemcpyAsync device to device
//   copy_small      copy of 128 MiB (fits the 256 MiB Infinity Cache): not an HBM number
//   read_span / read_claim[4|16] / read_win   the whole-file CRC's read pattern (readwin_k)
// Prints one JSON line per variant: bytes moved (read + written) / median time.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <string>
#include <vector>

typedef uint32_t u32;
typedef uint64_t u64;

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                     \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

template <int ILP, bool NTS, bool NTL>
__global__ __launch_bounds__(256) void copy_k(const uint4* __restrict__ s, uint4* __restrict__ d, u64 n16) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (ILP - 1) * stride < n16; i += ILP * stride) {
    uint4 v[ILP];
#pragma unroll
    for (int k = 0; k < ILP; k++) {
      if (NTL) {
        v[k].x = __builtin_nontemporal_load(&s[i + k * stride].x);
        v[k].y = __builtin_nontemporal_load(&s[i + k * stride].y);
        v[k].z = __builtin_nontemporal_load(&s[i + k * stride].z);
        v[k].w = __builtin_nontemporal_load(&s[i + k * stride].w);
      } else {
        v[k] = s[i + k * stride];
      }
    }
#pragma unroll
    for (int k = 0; k < ILP; k++) {
      if (NTS) {
        typedef u32 u32x4 __attribute__((ext_vector_type(4)));
        u32x4 t = {v[k].x, v[k].y, v[k].z, v[k].w};
        __builtin_nontemporal_store(t, reinterpret_cast<u32x4*>(&d[i + k * stride]));
      } else {
        d[i + k * stride] = v[k];
      }
    }
  }
  for (; i < n16; i += stride) d[i] = s[i];
}

// guide-style: one float4 per thread (or K consecutive per thread), a grid covering the buffer
template <int K, bool NT>
__global__ __launch_bounds__(256) void copy_flat_k(const uint4* __restrict__ s, uint4* __restrict__ d, u64 n16) {
  const u64 i0 = ((u64)blockIdx.x * blockDim.x) * K + threadIdx.x;
  uint4 v[K];
#pragma unroll
  for (int k = 0; k < K; k++)
    if (i0 + k * 256 < n16) v[k] = s[i0 + k * 256];
#pragma unroll
  for (int k = 0; k < K; k++)
    if (i0 + k * 256 < n16) {
      if (NT) {
        typedef u32 u32x4 __attribute__((ext_vector_type(4)));
        u32x4 t = {v[k].x, v[k].y, v[k].z, v[k].w};
        __builtin_nontemporal_store(t, reinterpret_cast<u32x4*>(&d[i0 + k * 256]));
      } else {
        d[i0 + k * 256] = v[k];
      }
    }
}

__global__ __launch_bounds__(256) void read_k(const uint4* __restrict__ s, u64 n16, u32* out) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  u32 acc = 0;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const uint4 a = s[i], b = s[i + stride], c = s[i + 2 * stride], e = s[i + 3 * stride];
    acc += a.x ^ b.y ^ c.z ^ e.w;
  }
  for (; i < n16; i += stride) acc += s[i].x;
  if (acc == 0x9E3779B9u) out[0] = acc;
}

// The whole-file CRC's read pattern without its fold (tpz_crc.hip crc_window_kernel): 8 KiB
// windows, lane l reads the 128-byte run 128 l bytes before the window end (8 x 16-B loads), the
// next window's loads issued before the current one is consumed.
//   MODE 0 read_span   persistent, 16 waves per CU, each wave a contiguous span of windows
//   MODE 1 read_claim  persistent, each wave claims CL windows at a time from one global counter
//   MODE 2 read_win    one window per wave, a grid covering the buffer (4 waves per workgroup)
//   MODE 3 read_ilCL   persistent, wave g takes spans k * waves + g of CL windows (static)
//   MODE 4 read_wgspan persistent, workgroup x a contiguous span, its waves every 16th window
template <int MODE, int CL>
__global__ __launch_bounds__(1024) void readwin_k(const uint8_t* __restrict__ s, u64 nwin, u32* ctr, u32* out) {
  const u32 lane = threadIdx.x & 63;
  const u64 wv = (u64)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const u64 nw = (u64)gridDim.x * (blockDim.x >> 6);
  u32 acc = 0;
  auto ld = [&](u64 g, uint4 (&v)[8]) {
    const uint8_t* p = s + (g << 13) + 8192 - 128 * (lane + 1);
#pragma unroll
    for (int c = 0; c < 8; c++) v[c] = *reinterpret_cast<const uint4*>(p + 16 * c);
  };
  auto use = [&](const uint4 (&v)[8]) {
#pragma unroll
    for (int c = 0; c < 8; c++) acc += v[c].x ^ v[c].y ^ v[c].z ^ v[c].w;
  };
  uint4 v[8], w[8];
  if (MODE == 2) {
    if (wv < nwin) { ld(wv, v); use(v); }
  } else if (MODE == 0) {
    const u64 per = (nwin + nw - 1) / nw, g0 = wv * per, g1 = min(nwin, g0 + per);
    if (g0 < g1) ld(g0, v);
    for (u64 g = g0; g < g1; g++) {
#pragma unroll
      for (int c = 0; c < 8; c++) w[c] = v[c];
      if (g + 1 < g1) ld(g + 1, v);
      use(w);
    }
  } else if (MODE == 3) {
    // static interleave: wave g takes spans k * nw + g of CL consecutive windows (no atomics)
    const u64 nsp = (nwin + CL - 1) / CL;
    u64 sp = wv, k = 0;
    if (sp < nsp) ld(sp * CL, v);
    while (sp < nsp) {
#pragma unroll
      for (int c = 0; c < 8; c++) w[c] = v[c];
      u64 gn;
      if (k + 1 < CL && sp * CL + k + 1 < nwin) { k++; gn = sp * CL + k; }
      else { sp += nw; k = 0; gn = sp * CL; }
      if (sp < nsp) ld(gn, v);
      use(w);
    }
  } else if (MODE == 4) {
    // workgroup spans: workgroup x owns a contiguous span of windows, its waves take every
    // (waves per workgroup)-th window of it (wave w: span start + k * W + w)
    const u64 W = blockDim.x >> 6, wid = threadIdx.x >> 6, nwg = gridDim.x;
    const u64 per = ((nwin + nwg - 1) / nwg + W - 1) / W * W;
    const u64 g0 = blockIdx.x * per + wid, g1 = min(nwin, (u64)(blockIdx.x + 1) * per);
    if (g0 < g1) ld(g0, v);
    for (u64 g = g0; g < g1; g += W) {
#pragma unroll
      for (int c = 0; c < 8; c++) w[c] = v[c];
      if (g + W < g1) ld(g + W, v);
      use(w);
    }
  } else {
    u32 base = 0;
    if (lane == 0) base = atomicAdd(ctr, 1u);
    u64 c0 = (u64)__builtin_amdgcn_readfirstlane(base) * CL;
    u32 nxt = 0;
    if (lane == 0) nxt = atomicAdd(ctr, 1u);
    u32 k = 0;
    if (c0 < nwin) ld(c0, v);
    while (c0 + k < nwin) {
#pragma unroll
      for (int c = 0; c < 8; c++) w[c] = v[c];
      u64 gn;
      if (k + 1 < CL) { gn = c0 + k + 1; k++; }
      else { c0 = (u64)__builtin_amdgcn_readfirstlane(nxt) * CL; k = 0; gn = c0; if (lane == 0) nxt = atomicAdd(ctr, 1u); }
      if (gn < nwin) ld(gn, v);
      use(w);
      if (gn >= nwin) break;
    }
  }
  if (acc == 0x9E3779B9u) out[16] = acc;
}

__global__ __launch_bounds__(256) void write_k(uint4* __restrict__ d, u64 n16) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
    d[i] = make_uint4((u32)i, 1, 2, 3);
}

// persistent: 16 waves per CU; wave w copies 4 KiB chunks w, w + W, ... (4 x 1 KiB per chunk,
// next chunk's loads in flight while this chunk's stores issue)
__global__ __launch_bounds__(1024) void wave4k_k(const uint4* __restrict__ s, uint4* __restrict__ d, u64 nchunks) {
  const u32 lane = threadIdx.x & 63;
  const u64 nw = (u64)gridDim.x * 16;
  u64 c = (u64)blockIdx.x * 16 + (threadIdx.x >> 6);
  uint4 v[4];
  if (c < nchunks)
#pragma unroll
    for (int q = 0; q < 4; q++) v[q] = s[c * 256 + q * 64 + lane];
  while (c < nchunks) {
    uint4 cur[4] = {v[0], v[1], v[2], v[3]};
    const u64 nx = c + nw;
    if (nx < nchunks)
#pragma unroll
      for (int q = 0; q < 4; q++) v[q] = s[nx * 256 + q * 64 + lane];
#pragma unroll
    for (int q = 0; q < 4; q++) d[c * 256 + q * 64 + lane] = cur[q];
    c = nx;
  }
}

// Persistent copies of 4 KiB chunks (64 lanes x 4 x 16 B), the next chunk's loads in flight while
// this chunk's stores issue, as the decode's wave path does. How a wave finds its chunks:
//   MODE 0  rows: wave (x, w) takes chunks k*W + 16x + w (the decode's row layout, static)
//   MODE 1  contiguous: wave g takes chunks [g*per, (g+1)*per)
//   MODE 2  dynamic: every chunk claimed from one global counter (claimed two ahead)
//   MODE 3  dynamic, 4 consecutive chunks per claim
//   MODE 4  per-XCD counters (blockIdx % 8), 16-chunk groups dealt round-robin to the XCDs, then
//           the other XCDs' counters once a wave's own runs out
//   MODE 5  semi-persistent: workgroup x takes the K rows of 16 chunks from 16 K x, then exits
//           (grid = nchunks / 16 K)
template <int MODE>
__global__ __launch_bounds__(1024) void persist_k(const uint4* __restrict__ s, uint4* __restrict__ d,
                                                 u64 nchunks, u32* ctr, u32 K = 0) {
  const u32 lane = threadIdx.x & 63, wv = threadIdx.x >> 6, wpg = blockDim.x >> 6;
  const u64 W = (u64)gridDim.x * wpg;
  const u64 g = (u64)blockIdx.x * wpg + wv;
  const u64 per = (nchunks + W - 1) / W;
  u64 k = 0;           // static modes: chunks taken so far
  u32 grp = 0, left = 0;  // MODE 3: current claim
  u32 xo = 0;          // MODE 4: counter offset being drained
  const u32 xcd = blockIdx.x & 7;
  const u64 ngroups = (nchunks + 15) >> 4;
  auto atom = [&](u32* c, u32 inc) -> u32 {
    u32 r = 0;
    if (lane == 0) r = atomicAdd(c, inc);
    return __builtin_amdgcn_readfirstlane(r);
  };
  auto next = [&]() -> u64 {
    if (MODE == 0) return (k++) * W + g;
    if (MODE == 5) { const u64 c = ((u64)blockIdx.x * K + k) * wpg + wv; return (k++ < K) ? c : ~0ull; }
    if (MODE == 1) { const u64 c = g * per + k; return (k++ < per) ? c : ~0ull; }
    if (MODE == 2) return atom(ctr, 1);
    if (MODE == 3) {
      if (!left) { grp = atom(ctr, 4); left = 4; }
      return (u64)grp + (4 - left--);
    }
    // MODE 4: XCD xc's groups are xc, xc + 8, ...; its counter counts chunks of those groups
    while (xo < 8) {
      const u32 xc = (xcd + xo) & 7;
      const u64 mine = (ngroups > xc) ? ((ngroups - xc + 7) >> 3) * 16 : 0;
      const u32 c = atom(ctr + 64 * xc, 1);
      if (c < mine) return ((u64)(c >> 4) * 8 + xc) * 16 + (c & 15);
      xo++;
    }
    return ~0ull;
  };
  u64 cur = next(), nxt = next();
  uint4 v[4];
  if (cur < nchunks)
#pragma unroll
    for (int q = 0; q < 4; q++) v[q] = s[cur * 256 + q * 64 + lane];
  while (cur < nchunks) {
    const u64 nn = next();
    uint4 w[4];
    if (nxt < nchunks)
#pragma unroll
      for (int q = 0; q < 4; q++) w[q] = s[nxt * 256 + q * 64 + lane];
#pragma unroll
    for (int q = 0; q < 4; q++) d[cur * 256 + q * 64 + lane] = v[q];
#pragma unroll
    for (int q = 0; q < 4; q++) v[q] = w[q];
    cur = nxt;
    nxt = nn;
  }
}

// rows (MODE 0) with two chunks' loads in flight while a chunk is stored; STORE_FIRST: the
// chunk's stores issue before the next chunk's loads
template <bool STORE_FIRST>
__global__ __launch_bounds__(1024) void rows2_k(const uint4* __restrict__ s, uint4* __restrict__ d, u64 nchunks) {
  const u32 lane = threadIdx.x & 63;
  const u64 W = (u64)gridDim.x * (blockDim.x >> 6);
  u64 c = (u64)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  uint4 a[4], b[4];
  if (c < nchunks)
#pragma unroll
    for (int q = 0; q < 4; q++) a[q] = s[c * 256 + q * 64 + lane];
  if (c + W < nchunks)
#pragma unroll
    for (int q = 0; q < 4; q++) b[q] = s[(c + W) * 256 + q * 64 + lane];
  while (c < nchunks) {
    uint4 n[4];
    const u64 c2 = c + 2 * W;
    if (STORE_FIRST) {
#pragma unroll
      for (int q = 0; q < 4; q++) d[c * 256 + q * 64 + lane] = a[q];
      if (c2 < nchunks)
#pragma unroll
        for (int q = 0; q < 4; q++) n[q] = s[c2 * 256 + q * 64 + lane];
    } else {
      if (c2 < nchunks)
#pragma unroll
        for (int q = 0; q < 4; q++) n[q] = s[c2 * 256 + q * 64 + lane];
#pragma unroll
      for (int q = 0; q < 4; q++) d[c * 256 + q * 64 + lane] = a[q];
    }
#pragma unroll
    for (int q = 0; q < 4; q++) { a[q] = b[q]; b[q] = n[q]; }
    c += W;
  }
}

// rows (MODE 0) with ping-pong buffers a / b (no register moves in the loop: a move of a
// register whose load is in flight waits for it): chunk c + W's loads in flight while chunk c
// is stored. Loads and stores past the end go through a buffer descriptor (no branches).
__device__ __forceinline__ void ld4(__amdgpu_buffer_rsrc_t r, u64 c, u32 lane, uint4 (&v)[4]) {
#pragma unroll
  for (int q = 0; q < 4; q++)
    v[q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, (u32)(c * 4096 + q * 1024 + lane * 16), 0, 0));
}
__device__ __forceinline__ void st4(__amdgpu_buffer_rsrc_t r, u64 c, u32 lane, const uint4 (&v)[4]) {
#pragma unroll
  for (int q = 0; q < 4; q++)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) u32, v[q]), r,
                                           (u32)(c * 4096 + q * 1024 + lane * 16), 0, 0);
}
// (offsets are u32: the buffers are viewed from a base per 4 GiB... the 4.36 GB case uses two
// halves, see the launch)
__global__ __launch_bounds__(1024) void pp_k(const uint8_t* __restrict__ s, uint8_t* __restrict__ d, u64 nchunks) {
  const u32 lane = threadIdx.x & 63;
  const u64 W = (u64)gridDim.x * (blockDim.x >> 6);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)s, (short)0, (int)(nchunks * 4096), 0x00020000);
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(d, (short)0, (int)(nchunks * 4096), 0x00020000);
  u64 c = (u64)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  uint4 a[4], b[4];
  ld4(rs, c, lane, a);
  while (c < nchunks) {
    ld4(rs, c + W, lane, b);
    st4(rd, c, lane, a);
    c += W;
    if (c >= nchunks) break;
    ld4(rs, c + W, lane, a);
    st4(rd, c, lane, b);
    c += W;
  }
}

// non-persistent: one wave per 4 KiB chunk (4 loads, 4 stores), 4 waves per workgroup
__global__ __launch_bounds__(256) void flat_w4k_k(const uint4* __restrict__ s, uint4* __restrict__ d, u64 nchunks) {
  const u32 lane = threadIdx.x & 63;
  const u64 c = (u64)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= nchunks) return;
  uint4 v[4];
#pragma unroll
  for (int q = 0; q < 4; q++) v[q] = s[c * 256 + q * 64 + lane];
#pragma unroll
  for (int q = 0; q < 4; q++) d[c * 256 + q * 64 + lane] = v[q];
}

int main(int argc, char** argv) {
  std::vector<std::string> vars;
  for (int i = 1; i < argc; i++) vars.push_back(argv[i]);
  if (vars.empty())
    vars = {"read", "write", "copy", "copy_ilp1", "copy_ilp8", "copy_nt", "copy_ntl", "copy_g4",
            "copy_g16", "copy_g32", "copy_wave4k", "memcpy", "copy_small", "read", "copy"};
  const u64 N = 4356833280ull;   // 2^20 x 4155 B, the 4k config's input
  const u64 PPN = 2147479552ull; // pp_*: 2 GiB - 4 KiB (32-bit buffer offsets), same pattern
  uint8_t *a, *b;
  u32* o;
  CHECK(hipMalloc(&a, N));
  CHECK(hipMalloc(&b, N));
  CHECK(hipMalloc(&o, 4096));
  CHECK(hipMemset(a, 0x5A, N));
  CHECK(hipMemset(b, 0, N));
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const u32 cus = prop.multiProcessorCount;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const u64 n16 = N / 16;
  const u64 small16 = (128ull << 20) / 16;
  for (const std::string& v : vars) {
    double moved = 2.0 * N;
    auto launch = [&]() {
      const uint4* s = (const uint4*)a;
      uint4* d = (uint4*)b;
      if (v == "read") { read_k<<<cus * 8, 256>>>(s, n16, o); }
      else if (v == "write") { write_k<<<cus * 8, 256>>>(d, n16); }
      else if (v == "copy") copy_k<4, false, false><<<cus * 8, 256>>>(s, d, n16);
      else if (v == "copy_ilp1") copy_k<1, false, false><<<cus * 8, 256>>>(s, d, n16);
      else if (v == "copy_ilp8") copy_k<8, false, false><<<cus * 8, 256>>>(s, d, n16);
      else if (v == "copy_nt") copy_k<4, true, false><<<cus * 8, 256>>>(s, d, n16);
      else if (v == "copy_ntl") copy_k<4, true, true><<<cus * 8, 256>>>(s, d, n16);
      else if (v == "copy_g4") copy_k<4, false, false><<<cus * 4, 256>>>(s, d, n16);
      else if (v == "copy_g16") copy_k<4, false, false><<<cus * 16, 256>>>(s, d, n16);
      else if (v == "copy_g32") copy_k<4, false, false><<<cus * 32, 256>>>(s, d, n16);
      else if (v == "copy_wave4k") wave4k_k<<<cus, 1024>>>(s, d, N / 4096);
      else if (v == "copy_flat") copy_flat_k<1, false><<<(u32)((n16 + 255) / 256), 256>>>(s, d, n16);
      else if (v == "copy_flat4") copy_flat_k<4, false><<<(u32)((n16 + 1023) / 1024), 256>>>(s, d, n16);
      else if (v == "copy_flat_nt") copy_flat_k<1, true><<<(u32)((n16 + 255) / 256), 256>>>(s, d, n16);
      else if (v == "p_rows") persist_k<0><<<cus, 1024>>>(s, d, N / 4096, o);
      else if (v == "p_rows8") persist_k<0><<<cus, 512>>>(s, d, N / 4096, o);
      else if (v == "p_rows32") persist_k<0><<<cus * 2, 1024>>>(s, d, N / 4096, o);
      else if (v == "p_contig") persist_k<1><<<cus, 1024>>>(s, d, N / 4096, o);
      else if (v == "p_dyn") persist_k<2><<<cus, 1024>>>(s, d, N / 4096, o);
      else if (v == "p_dyn32") persist_k<2><<<cus * 2, 1024>>>(s, d, N / 4096, o);
      else if (v == "p_dyn4") persist_k<3><<<cus, 1024>>>(s, d, N / 4096, o);
      else if (v == "p_xcd") persist_k<4><<<cus, 1024>>>(s, d, N / 4096, o);
      else if (v == "p_semi4") persist_k<5><<<(u32)(N / 4096 / 64), 1024>>>(s, d, N / 4096, o, 4);
      else if (v == "p_semi16") persist_k<5><<<(u32)(N / 4096 / 256), 1024>>>(s, d, N / 4096, o, 16);
      else if (v == "p_semi64") persist_k<5><<<(u32)(N / 4096 / 1024), 1024>>>(s, d, N / 4096, o, 64);
      else if (v == "p_semi16_256") persist_k<5><<<(u32)(N / 4096 / 64), 256>>>(s, d, N / 4096, o, 16);
      else if (v == "p_rows_256x4") persist_k<0><<<cus * 4, 256>>>(s, d, N / 4096, o);
      else if (v == "p_rows2") rows2_k<false><<<cus, 1024>>>(s, d, N / 4096);
      else if (v == "p_rows2s") rows2_k<true><<<cus, 1024>>>(s, d, N / 4096);
      else if (v == "p_rows2_8") rows2_k<false><<<cus, 512>>>(s, d, N / 4096);
      else if (v == "pp") pp_k<<<cus, 1024>>>(a, b, PPN / 4096);
      else if (v == "pp8") pp_k<<<cus, 512>>>(a, b, PPN / 4096);
      else if (v == "pp32") pp_k<<<cus * 2, 1024>>>(a, b, PPN / 4096);
      else if (v == "pp_flat") flat_w4k_k<<<(u32)(PPN / 4096 / 4), 256>>>(s, d, PPN / 4096);
      else if (v == "flat_w4k") flat_w4k_k<<<(u32)(N / 4096 / 4), 256>>>(s, d, N / 4096);
      else if (v == "read_span") readwin_k<0, 1><<<cus, 1024>>>(a, N >> 13, o, o);
      else if (v == "read_claim") readwin_k<1, 1><<<cus, 1024>>>(a, N >> 13, o, o);
      else if (v == "read_claim4") readwin_k<1, 4><<<cus, 1024>>>(a, N >> 13, o, o);
      else if (v == "read_claim16") readwin_k<1, 16><<<cus, 1024>>>(a, N >> 13, o, o);
      else if (v == "read_il1") readwin_k<3, 1><<<cus, 1024>>>(a, N >> 13, o, o);
      else if (v == "read_il4") readwin_k<3, 4><<<cus, 1024>>>(a, N >> 13, o, o);
      else if (v == "read_il16") readwin_k<3, 16><<<cus, 1024>>>(a, N >> 13, o, o);
      else if (v == "read_il64") readwin_k<3, 64><<<cus, 1024>>>(a, N >> 13, o, o);
      else if (v == "read_il16x2") readwin_k<3, 16><<<2 * cus, 1024>>>(a, N >> 13, o, o);
      else if (v == "read_wgspan") readwin_k<4, 1><<<cus, 1024>>>(a, N >> 13, o, o);
      else if (v == "read_wgspan8") readwin_k<4, 1><<<cus, 512>>>(a, N >> 13, o, o);
      else if (v == "read_wgspan2x") readwin_k<4, 1><<<2 * cus, 1024>>>(a, N >> 13, o, o);
      else if (v == "read_win") readwin_k<2, 1><<<(u32)((N >> 13) / 4), 256>>>(a, N >> 13, o, o);
      else if (v == "memcpy") (void)hipMemcpyAsync(b, a, N, hipMemcpyDeviceToDevice, 0);
      else if (v == "copy_small") copy_k<4, false, false><<<cus * 8, 256>>>(s, d, small16);
    };
    if (v == "read" || v == "write" || v.rfind("read_", 0) == 0) moved = (double)N;
    if (v.rfind("pp", 0) == 0) moved = 2.0 * PPN;
    if (v == "copy_small") moved = 2.0 * (128ull << 20);
    for (int w = 0; w < 3; w++) { CHECK(hipMemsetAsync(o, 0, 4096)); launch(); }
    CHECK(hipDeviceSynchronize());
    const int reps = 15;
    std::vector<float> ms;
    for (int r = 0; r < reps; r++) {
      CHECK(hipMemsetAsync(o, 0, 4096));
      CHECK(hipEventRecord(e0));
      launch();
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float t;
      CHECK(hipEventElapsedTime(&t, e0, e1));
      ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    const float med = ms[reps / 2];
    printf("{\"variant\": \"%s\", \"bytes\": %.0f, \"ms_median\": %.4f, \"ms_min\": %.4f, \"tb_s\": %.3f}\n",
           v.c_str(), moved, med, ms[0], moved / (med * 1e-3) / 1e12);
    fflush(stdout);
  }
  return 0;
}
