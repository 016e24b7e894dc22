// ubench_pipe.hip — does a persistent loop that never waits for its own stores move the decode's
// bytes at the one-shot copy's rate? (diagnostic, GPU box)
//
// Every variant copies the 4k config's 4.36 GB (4 KiB chunks) once:
//   flat      one 16-byte piece per thread, 256-thread workgroups, the grid covers the buffer
//   w4k       one chunk per wave, 4 waves per workgroup, non-persistent
//   pipe      persistent, 16 waves per CU (one 1024-thread workgroup), a wave claims chunks in
//             rows; chunk i+1's four loads are issued before chunk i's four stores and waited for
//             at the top of the next iteration: every iteration issues the same VMEM ops, so the
//             compiler's wait is vmcnt(4) (the previous stores stay in flight)
//   pipe_lds  pipe, the chunk staged through a per-wave LDS window (ds_write / ds_read) as the
//             decode does
//   pipe_meta pipe_lds plus three small per-chunk stores (status u8, count u32, crc u32) and one
//             512-B ends store, as the decode writes
//   pipe_w0   pipe_lds with a full drain (vmcnt(0)) at the top: the previous chunk's stores are
//             waited for (the decode's loop today)
//   pipe2     pipe_lds with two chunks in flight (loads two iterations ahead, ping-pong buffers)
//   pipe_meta3   pipe_lds plus the three per-chunk status / count / crc stores (lane 0, the other
//                lanes' offsets past the descriptor), no ends store
//   pipe_meta3x  the same three stores exec-masked to lane 0
//   pipe_meta1   one store instruction, lanes 0-2 to the three arrays
//   pipe_metarow the three arrays written per row of 16 chunks (wave 0, lanes 0-15)
//   pipe_meta8   one packed 8-byte record per chunk (lane 0): a row's 16 records fill one line
//   (profiles/r5/ubench_meta.jsonl: 1.59 / 1.77 / 1.77 / 1.81 / 1.66 ms for pipe_lds / meta3 /
//   meta3x / meta1 / metarow: each small store is a write request of its own whatever its lane
//   count; batching per row recovers two thirds in this kernel, but not in the decode,
//   profiles/r5/meta_rows_ab.jsonl)
//
//     hipcc -O3 --offload-arch=gfx950 -o tools/ubench_pipe tools/ubench_pipe.hip
//     tools/ubench_pipe [variant ...]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <string>
#include <vector>

typedef uint32_t u32;
typedef uint64_t u64;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                         \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                          \
    }                                                                    \
  } while (0)

__global__ __launch_bounds__(256) void flat_k(const uint4* __restrict__ s, uint4* __restrict__ d, u64 n16) {
  const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
  if (i < n16) d[i] = s[i];
}

__global__ __launch_bounds__(256) void w4k_k(const uint4* __restrict__ s, uint4* __restrict__ d, u64 nchunks) {
  const u32 lane = threadIdx.x & 63;
  const u64 c = (u64)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= nchunks) return;
  uint4 v[4];
#pragma unroll
  for (int q = 0; q < 4; q++) v[q] = s[c * 256 + q * 64 + lane];
#pragma unroll
  for (int q = 0; q < 4; q++) d[c * 256 + q * 64 + lane] = v[q];
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, u64 bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)(bytes > 0x7FFFFFF0ull ? 0x7FFFFFF0ull : bytes), 0x00020000);
}

// MODE 0 pipe, 1 pipe_lds, 2 pipe_meta, 3 pipe_w0
template <int MODE>
__global__ __launch_bounds__(1024) void pipe_k(const uint8_t* __restrict__ s, uint8_t* __restrict__ d,
                                               uint8_t* __restrict__ meta, u64 nchunks) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[16 * 4096];
  const u32 lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 wpg = blockDim.x >> 6;
  const u64 W = (u64)gridDim.x * wpg;
  u64 c = (u64)blockIdx.x * wpg + wv;
  uint8_t* win = lds + wv * 4096;
  uint4 v[4];
  auto load = [&](u64 cc) {
    // chunks past the end read through a zero-length descriptor (no branch, same op count)
    const __amdgpu_buffer_rsrc_t r = rsrc(s + (cc < nchunks ? cc : 0) * 4096, cc < nchunks ? 4096 : 0);
#pragma unroll
    for (int q = 0; q < 4; q++)
      v[q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, q * 1024 + lane * 16, 0, 0));
  };
  if (c >= nchunks) return;
  load(c);
  __builtin_amdgcn_sched_barrier(0);
  // as many VMEM ops after the first loads as every iteration issues after its loads (the four
  // stores, to a zero-length descriptor: nothing is written), so that the loop-top wait, which must
  // hold for the entry path too, is vmcnt(4) and not vmcnt(0)
  {
    const __amdgpu_buffer_rsrc_t rz = rsrc(d, 0);
#pragma unroll
    for (int q = 0; q < (MODE == 2 ? 8 : MODE == 6 ? 7 : MODE == 7 ? 5 : MODE == 8 ? 7 : MODE == 9 ? 5 : MODE == 11 ? 5 : 4); q++)
      __builtin_amdgcn_raw_buffer_store_b32(0u, rz, q * 256, 0, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
  do {
    if (MODE == 3) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint4 o[4];
    if (MODE == 0) {
#pragma unroll
      for (int q = 0; q < 4; q++) o[q] = v[q];
    } else {
#pragma unroll
      for (int q = 0; q < 4; q++) *reinterpret_cast<uint4*>(win + q * 1024 + lane * 16) = v[q];
    }
    const u64 cn = c + W;
    load(cn);                                      // next chunk's loads before this chunk's stores
    if (MODE != 0) {
      __builtin_amdgcn_wave_barrier();
      // read back at an offset (a rotation within the window), as the decode's gathers do
#pragma unroll
      for (int q = 0; q < 4; q++) o[q] = *reinterpret_cast<const uint4*>(win + ((q * 1024 + lane * 16 + 16) & 4095));
    }
    const __amdgpu_buffer_rsrc_t rd = rsrc(d + c * 4096, MODE == 5 ? 0 : 4096);
#pragma unroll
    for (int q = 0; q < 4; q++)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o[q]), rd, q * 1024 + lane * 16, 0,
                                             MODE == 4 ? 2 : 0);
    if (MODE == 2 || MODE == 6) {
      const __amdgpu_buffer_rsrc_t rm = rsrc(meta, 0x7FFFFFF0ull);
      const bool l0 = lane == 0;
      // status u8, count u32, crc u32 (three arrays, one entry per chunk)
      __builtin_amdgcn_raw_buffer_store_b8((uint8_t)c, rm, l0 ? (u32)c : 0x7FFFFFF8u, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32((u32)c, rm, l0 ? (u32)(0x200000 + 4 * c) : 0x7FFFFFF8u, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32((u32)c, rm, l0 ? (u32)(0x800000 + 4 * c) : 0x7FFFFFF8u, 0, 0);
    }
    if (MODE == 8 && lane == 0) {   // the three small stores from lane 0 alone (exec-masked)
      const __amdgpu_buffer_rsrc_t rm = rsrc(meta, 0x7FFFFFF0ull);
      __builtin_amdgcn_raw_buffer_store_b8((uint8_t)c, rm, (u32)c, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32((u32)c, rm, (u32)(0x200000 + 4 * c), 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32((u32)c, rm, (u32)(0x800000 + 4 * c), 0, 0);
    }
    if (MODE == 9 && lane < 3) {    // one store instruction, lanes 0-2 to the three arrays
      const __amdgpu_buffer_rsrc_t rm = rsrc(meta, 0x7FFFFFF0ull);
      __builtin_amdgcn_raw_buffer_store_b32((u32)c, rm, lane == 0 ? (u32)(4 * c) : (u32)((lane == 1 ? 0x200000 : 0x800000) + 4 * c), 0, 0);
    }
    if (MODE == 10 && wv == 0) {   // a row's metadata at once: wave 0, lanes 0-15, 3 stores
      const __amdgpu_buffer_rsrc_t rm = rsrc(meta, 0x7FFFFFF0ull);
      const u32 i = (u32)c + lane;   // (wave 0's chunk is the row's first)
      const bool on = lane < 16;
      __builtin_amdgcn_raw_buffer_store_b8((uint8_t)i, rm, on ? i : 0x7FFFFFF8u, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32(i, rm, on ? (u32)(0x200000 + 4 * i) : 0x7FFFFFF8u, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32(i, rm, on ? (u32)(0x800000 + 4 * i) : 0x7FFFFFF8u, 0, 0);
    }
    if (MODE == 11) {   // one packed 8-byte record per chunk (status | count | crc): a row of 16
                        // chunks fills one 128-B line, written by one workgroup
      const __amdgpu_buffer_rsrc_t rm = rsrc(meta, 0x7FFFFFF0ull);
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) u32, make_uint2((u32)c, (u32)c)),
                                            rm, lane == 0 ? (u32)(8 * c) : 0x7FFFFFF8u, 0, 0);
    }
    if (MODE == 2 || MODE == 7) {
      // one 512-B ends store per chunk, into an ends region of its own (chunk c's at 512 c of d,
      // past the copied data)
      const __amdgpu_buffer_rsrc_t re = rsrc(d + nchunks * 4096 + c * 512, 512);
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) u32, make_uint2(lane, (u32)c)),
                                            re, 8 * lane, 0, 0);
    }
    c = cn;
  } while (c < nchunks);
}

// 4 KiB chunks with the piece loads and stores interleaved: piece q of chunk c is stored, then
// piece q of the next chunk loaded (each load has a whole iteration to arrive)
__global__ __launch_bounds__(1024) void pipeil_k(const uint8_t* __restrict__ s, uint8_t* __restrict__ d, u64 nchunks) {
  const u32 lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u64 W = (u64)gridDim.x * 16;
  u64 c = (u64)blockIdx.x * 16 + wv;
  if (c >= nchunks) return;
  uint4 v[4];
  auto ld = [&](u64 cc, int q) {
    const __amdgpu_buffer_rsrc_t r = rsrc(s + (cc < nchunks ? cc : 0) * 4096, cc < nchunks ? 4096 : 0);
    v[q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, q * 1024 + lane * 16, 0, 0));
  };
#pragma unroll
  for (int q = 0; q < 4; q++) ld(c, q);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int q = 0; q < 4; q++) __builtin_amdgcn_raw_buffer_store_b32(0u, rsrc(d, 0), q * 256, 0, 0);
  __builtin_amdgcn_sched_barrier(0);
  do {
    const u64 cn = c + W;
    const __amdgpu_buffer_rsrc_t rd = rsrc(d + c * 4096, 4096);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint4 o = v[q];
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rd, q * 1024 + lane * 16, 0, 0);
      ld(cn, q);
      __builtin_amdgcn_sched_barrier(0);
    }
    c = cn;
  } while (c < nchunks);
}

// pipe_lds with the workgroup's rows of 16 chunks claimed from one global counter (one atomic
// per row, its chunks handed to the waves through LDS): every workgroup works near the others,
// the chunks in flight stay within a narrow window of the buffer
__global__ __launch_bounds__(1024) void pipedyn_k(const uint8_t* __restrict__ s, uint8_t* __restrict__ d,
                                                  u32* ctr, u64 nchunks) {
  __shared__ u32 row_of[2];
  __shared__ u32 taken;
  const u32 lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u64 nrows = (nchunks + 15) / 16;
  // every wave takes chunk wv of row r (one row per workgroup iteration): a workgroup barrier per
  // row hands the next row's index to all waves
  if (threadIdx.x == 0) row_of[0] = atomicAdd(ctr, 1u);
  __syncthreads();
  u64 r = row_of[0];
  uint4 v[4];
  auto load = [&](u64 cc) {
    const __amdgpu_buffer_rsrc_t rr = rsrc(s + (cc < nchunks ? cc : 0) * 4096, cc < nchunks ? 4096 : 0);
#pragma unroll
    for (int q = 0; q < 4; q++)
      v[q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rr, q * 1024 + lane * 16, 0, 0));
  };
  load(r * 16 + wv);
  int flip = 0;
  while (r < nrows) {
    if (threadIdx.x == 0) row_of[flip ^ 1] = atomicAdd(ctr, 1u);
    __syncthreads();
    const u64 rn = row_of[flip ^ 1];
    flip ^= 1;
    uint4 o[4];
#pragma unroll
    for (int q = 0; q < 4; q++) o[q] = v[q];
    load(rn * 16 + wv);
    const u64 c = r * 16 + wv;
    const __amdgpu_buffer_rsrc_t rd = rsrc(d + (c < nchunks ? c : 0) * 4096, c < nchunks ? 4096 : 0);
#pragma unroll
    for (int q = 0; q < 4; q++)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o[q]), rd, q * 1024 + lane * 16, 0, 0);
    r = rn;
  }
  (void)taken;
}

// 1 KiB pieces: each iteration one 16-byte load and one store per lane (wave w of workgroup x
// takes piece (k * grid + x) * 16 + w), the next piece's load before this piece's store
__global__ __launch_bounds__(1024) void pipe1k_k(const uint8_t* __restrict__ s, uint8_t* __restrict__ d, u64 npieces) {
  const u32 lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u64 W = (u64)gridDim.x * 16;
  u64 c = (u64)blockIdx.x * 16 + wv;
  if (c >= npieces) return;
  auto load = [&](u64 cc) -> uint4 {
    const __amdgpu_buffer_rsrc_t r = rsrc(s + (cc < npieces ? cc : 0) * 1024, cc < npieces ? 1024 : 0);
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, 0, 0));
  };
  uint4 v = load(c);
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_raw_buffer_store_b32(0u, rsrc(d, 0), 0, 0, 0);
  __builtin_amdgcn_sched_barrier(0);
  do {
    const uint4 o = v;
    const u64 cn = c + W;
    v = load(cn);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rsrc(d + c * 1024, 1024), lane * 16, 0, 0);
    c = cn;
  } while (c < npieces);
}

// two chunks in flight: a / b ping-pong, loads two iterations ahead
__global__ __launch_bounds__(1024) void pipe2_k(const uint8_t* __restrict__ s, uint8_t* __restrict__ d, u64 nchunks) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[16 * 4096];
  const u32 lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u64 W = (u64)gridDim.x * 16;
  u64 c = (u64)blockIdx.x * 16 + wv;
  uint8_t* win = lds + wv * 4096;
  uint4 a[4], b[4];
  auto load = [&](u64 cc, uint4 (&v)[4]) {
    const __amdgpu_buffer_rsrc_t r = rsrc(s + (cc < nchunks ? cc : 0) * 4096, cc < nchunks ? 4096 : 0);
#pragma unroll
    for (int q = 0; q < 4; q++)
      v[q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, q * 1024 + lane * 16, 0, 0));
  };
  auto body = [&](u64 cc, uint4 (&v)[4]) {
#pragma unroll
    for (int q = 0; q < 4; q++) *reinterpret_cast<uint4*>(win + q * 1024 + lane * 16) = v[q];
    load(cc + 2 * W, v);
    __builtin_amdgcn_wave_barrier();
    uint4 o[4];
#pragma unroll
    for (int q = 0; q < 4; q++) o[q] = *reinterpret_cast<const uint4*>(win + ((q * 1024 + lane * 16 + 16) & 4095));
    const __amdgpu_buffer_rsrc_t rd = rsrc(d + cc * 4096, 4096);
#pragma unroll
    for (int q = 0; q < 4; q++)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o[q]), rd, q * 1024 + lane * 16, 0, 0);
  };
  if (c >= nchunks) return;
  load(c, a);
  load(c + W, b);
  __builtin_amdgcn_sched_barrier(0);
  {
    const __amdgpu_buffer_rsrc_t rz = rsrc(d, 0);
#pragma unroll
    for (int q = 0; q < 8; q++) __builtin_amdgcn_raw_buffer_store_b32(0u, rz, q * 256, 0, 0);
  }
  do {
    body(c, a);
    c += W;
    if (c >= nchunks) break;
    body(c, b);
    c += W;
  } while (c < nchunks);
}

int main(int argc, char** argv) {
  std::vector<std::string> vars;
  for (int i = 1; i < argc; i++) vars.push_back(argv[i]);
  if (vars.empty()) vars = {"flat", "w4k", "pipe", "pipe_lds", "pipe_meta", "pipe_w0", "pipe2", "pipe_nt", "pipe_rd",
                            "pipe32", "pipe1k", "pipe1k32", "pipe_512", "pipe_il", "pipe8", "pipe_dyn", "flat",
                            "pipe_lds"};
  const u64 N = 4356833280ull;   // the 4k config's input bytes
  const u64 nch = N / 4096;
  uint8_t *a, *b, *m;
  CHECK(hipMalloc(&a, N));
  CHECK(hipMalloc(&b, N + (N / 4096) * 512));
  CHECK(hipMalloc(&m, 64u << 20));
  CHECK(hipMemset(a, 0x5A, N));
  CHECK(hipMemset(b, 0, N));
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const u32 cus = prop.multiProcessorCount;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (const std::string& v : vars) {
    auto launch = [&]() {
      if (v == "flat") flat_k<<<(u32)(N / 16 / 256), 256>>>((const uint4*)a, (uint4*)b, N / 16);
      else if (v == "w4k") w4k_k<<<(u32)(nch / 4), 256>>>((const uint4*)a, (uint4*)b, nch);
      else if (v == "pipe") pipe_k<0><<<cus, 1024>>>(a, b, m, nch);
      else if (v == "pipe_lds") pipe_k<1><<<cus, 1024>>>(a, b, m, nch);
      else if (v == "pipe_meta") pipe_k<2><<<cus, 1024>>>(a, b, m, nch);
      else if (v == "pipe_w0") pipe_k<3><<<cus, 1024>>>(a, b, m, nch);
      else if (v == "pipe2") pipe2_k<<<cus, 1024>>>(a, b, nch);
      else if (v == "pipe_nt") pipe_k<4><<<cus, 1024>>>(a, b, m, nch);
      else if (v == "pipe_il") pipeil_k<<<cus, 1024>>>(a, b, nch);
      else if (v == "pipe_meta3") pipe_k<6><<<cus, 1024>>>(a, b, m, nch);
      else if (v == "pipe_ends") pipe_k<7><<<cus, 1024>>>(a, b, m, nch);
      else if (v == "pipe_meta3x") pipe_k<8><<<cus, 1024>>>(a, b, m, nch);
      else if (v == "pipe_meta1") pipe_k<9><<<cus, 1024>>>(a, b, m, nch);
      else if (v == "pipe_metarow") pipe_k<10><<<cus, 1024>>>(a, b, m, nch);
      else if (v == "pipe_meta8") pipe_k<11><<<cus, 1024>>>(a, b, m, nch);
      else if (v == "pipe8") pipe_k<1><<<cus, 512>>>(a, b, m, nch);
      else if (v == "pipe_dyn") { (void)hipMemsetAsync(m, 0, 4); pipedyn_k<<<cus, 1024>>>(a, b, (u32*)m, nch); }
      else if (v == "pipe_rd") pipe_k<5><<<cus, 1024>>>(a, b, m, nch);
      else if (v == "pipe32") pipe_k<1><<<2 * cus, 1024>>>(a, b, m, nch);
      else if (v == "pipe1k") pipe1k_k<<<cus, 1024>>>(a, b, N / 1024);
      else if (v == "pipe1k32") pipe1k_k<<<2 * cus, 1024>>>(a, b, N / 1024);
      else if (v == "pipe_512") pipe_k<1><<<cus, 1024>>>(a, b, m, nch / 2);
    };
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
    const double moved = v == "pipe_rd" ? (double)N : v == "pipe_512" ? (double)N : 2.0 * N;
    printf("{\"variant\": \"%s\", \"ms_median\": %.4f, \"ms_min\": %.4f, \"tb_s\": %.3f}\n", v.c_str(), med,
           ms[0], moved / (med * 1e-3) / 1e12);
    fflush(stdout);
  }
  return 0;
}
