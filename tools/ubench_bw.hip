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

int main(int argc, char** argv) {
  std::vector<std::string> vars;
  for (int i = 1; i < argc; i++) vars.push_back(argv[i]);
  if (vars.empty())
    vars = {"read", "write", "copy", "copy_ilp1", "copy_ilp8", "copy_nt", "copy_ntl", "copy_g4",
            "copy_g16", "copy_g32", "copy_wave4k", "memcpy", "copy_small", "read", "copy"};
  const u64 N = 4356833280ull;   // 2^20 x 4155 B, the 4k config's input
  uint8_t *a, *b;
  u32* o;
  CHECK(hipMalloc(&a, N));
  CHECK(hipMalloc(&b, N));
  CHECK(hipMalloc(&o, 4));
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
      else if (v == "memcpy") (void)hipMemcpyAsync(b, a, N, hipMemcpyDeviceToDevice, 0);
      else if (v == "copy_small") copy_k<4, false, false><<<cus * 8, 256>>>(s, d, small16);
    };
    if (v == "read" || v == "write") moved = (double)N;
    if (v == "copy_small") moved = 2.0 * (128ull << 20);
    for (int w = 0; w < 3; w++) launch();
    CHECK(hipDeviceSynchronize());
    const int reps = 15;
    std::vector<float> ms;
    for (int r = 0; r < reps; r++) {
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
