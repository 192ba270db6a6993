// terasort.hip — TeraSort-style key/value sort kernels (gfx950).
//
// Records are the TeraSort/gensort layout: 100 bytes = 10-byte key + 90-byte
// value, stored row-major in HBM (4-byte aligned: 25 u32 words per record).
// The BASELINE "TeraSort-style 10 GB key/value sort (radix sort + all-to-all)"
// workload; the MapReduce shape is an identity map, a range partitioner from
// sampled splitters (TeraSort's TotalOrderPartitioner) and an identity reduce —
// the reference's shuffle + per-partition key sort.
//
//   ts_gen     : TeraGen analogue — record r of a seed, computed word-parallel
//                (thread per u32) so the 10 GB write is coalesced;
//   ts_keys    : (hi, lo) sort words: key bytes 0-7 big-endian, bytes 8-9;
//   ts_checksum: order-independent sum of per-record 64-bit hashes;
//   ts_unsorted: number of adjacent (hi, lo) pairs out of order.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "mr_common.h"

namespace mr {
namespace ts {

constexpr int WORDS = 25;  // 100-byte records

__device__ __forceinline__ u64 splitmix(u64 x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// byte b (0..99) of record r
__device__ __forceinline__ u32 rec_byte(u64 seed, u64 r, u32 b) {
  if (b < 8) return (u32)(splitmix(seed ^ (r * 2 + 0)) >> (56 - 8 * b)) & 0xFFu;
  if (b < 10) return (u32)(splitmix(seed ^ (r * 2 + 1)) >> (56 - 8 * (b - 8))) & 0xFFu;
  if (b < 18) return (u32)(r >> (8 * (b - 10))) & 0xFFu;  // record number, little-endian
  return (u32)((r * 31u + b * 7u) & 0x3Fu) + 0x30u;       // printable filler
}

__global__ void ts_gen_kernel(u32* __restrict__ out, u64 n, u64 first, u64 seed) {
  const u64 nw = n * WORDS;
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 w = (u64)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += stride) {
    const u64 r = w / WORDS;
    const u32 j = (u32)(w - r * WORDS);
    const u64 gr = first + r;
    u32 v;
    if (j < 5) {
      v = 0;
      for (u32 k = 0; k < 4; ++k) v |= rec_byte(seed, gr, 4 * j + k) << (8 * k);
    } else {
      v = 0;
      for (u32 k = 0; k < 4; ++k) v |= ((u32)((gr * 31u + (4 * j + k) * 7u) & 0x3Fu) + 0x30u) << (8 * k);
    }
    out[w] = v;
  }
}

// Sort words of each record; with `ghist` also the radix sort's digit
// histograms of the top 32 bits of hi (digits 4..7 of the [8][256] layout of
// sort.hip's rs_ghist8_kernel), so the sort skips its histogram pass over the
// 100 M keys (0.27 ms per 10 GB).  256 threads per block.
__global__ void __launch_bounds__(256) ts_keys_kernel(const u32* __restrict__ rec, u64 n, u64* __restrict__ hi,
                                                      u64* __restrict__ lo, u32* __restrict__ ghist) {
  __shared__ u32 h[4][256];
  const int t = threadIdx.x;
  if (ghist) {
#pragma unroll
    for (int b = 0; b < 4; ++b) h[b][t] = 0;
    __syncthreads();
  }
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + t; i < n; i += stride) {
    const u32* p = rec + i * WORDS;
    const u32 w0 = p[0], w1 = p[1], w2 = p[2];
    const u32 top = __builtin_bswap32(w0);
    hi[i] = ((u64)top << 32) | (u64)__builtin_bswap32(w1);
    lo[i] = (u64)(((w2 & 0xFFu) << 8) | ((w2 >> 8) & 0xFFu));
    if (ghist) {
#pragma unroll
      for (int b = 0; b < 4; ++b) atomicAdd(&h[b][(top >> (8 * b)) & 0xFFu], 1u);
    }
  }
  if (ghist) {
    __syncthreads();
#pragma unroll
    for (int b = 0; b < 4; ++b)
      if (h[b][t]) atomicAdd(&ghist[(4 + b) * 256 + t], h[b][t]);
  }
}

__global__ void __launch_bounds__(256) ts_checksum_kernel(const u32* __restrict__ rec, u64 n,
                                                          unsigned long long* __restrict__ out) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  u64 acc = 0;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const u32* p = rec + i * WORDS;
    u64 h = 0x243F6A8885A308D3ull;
    for (int j = 0; j < WORDS; ++j) h = fmix64(h ^ p[j]) + (u64)j;
    acc += h;
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)acc);
}

__global__ void __launch_bounds__(256) ts_unsorted_kernel(const u64* __restrict__ hi, const u64* __restrict__ lo,
                                                          u64 n, unsigned long long* __restrict__ out) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  u64 bad = 0;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x + 1; i < n; i += stride) {
    const u64 a = hi[i - 1], b = hi[i];
    bad += (a > b) || (a == b && lo[i - 1] > lo[i]);
  }
  for (int o = 32; o > 0; o >>= 1) bad += __shfl_xor(bad, o);
  if ((threadIdx.x & 63) == 0 && bad) atomicAdd(out, (unsigned long long)bad);
}

}  // namespace ts
}  // namespace mr

using namespace mr;

static inline unsigned ts_grid(u64 n, unsigned cap = 8192) {
  u64 g = (n + 255) / 256;
  return (unsigned)(g < 1 ? 1 : (g > cap ? cap : g));
}

extern "C" {

int mr_ts_gen(void* out, u64 n, u64 first, u64 seed, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(ts::ts_gen_kernel, dim3(ts_grid(n * ts::WORDS)), dim3(256), 0, s, (u32*)out, n, first, seed);
  return (int)hipGetLastError();
}

// ghist: null, or a zeroed u32[8][256] that receives the histograms of the
// digits 4..7 of hi (the top-32-bit sort of sort_perm)
int mr_ts_keys(const void* rec, u64 n, void* hi, void* lo, void* ghist, hipStream_t s) {
  if (n == 0) return 0;
  // with histograms: at most 2048 blocks (each adds its 1024 bins to the
  // same 1024 global counters)
  hipLaunchKernelGGL(ts::ts_keys_kernel, dim3(ts_grid(n, ghist ? 2048 : 8192)), dim3(256), 0, s, (const u32*)rec, n,
                     (u64*)hi, (u64*)lo, (u32*)ghist);
  return (int)hipGetLastError();
}

int mr_ts_checksum(const void* rec, u64 n, void* out, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(ts::ts_checksum_kernel, dim3(ts_grid(n, 2048)), dim3(256), 0, s, (const u32*)rec, n,
                     (unsigned long long*)out);
  return (int)hipGetLastError();
}

int mr_ts_unsorted(const void* hi, const void* lo, u64 n, void* out, hipStream_t s) {
  if (n < 2) return 0;
  hipLaunchKernelGGL(ts::ts_unsorted_kernel, dim3(ts_grid(n, 2048)), dim3(256), 0, s, (const u64*)hi,
                     (const u64*)lo, n, (unsigned long long*)out);
  return (int)hipGetLastError();
}

}  // extern "C"
