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
//   ts_dest    : destination rank = #splitters <= hi (splitters in LDS);
//   ts_gather  : out row i = in row perm[i], one thread per u32 word;
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

__global__ void ts_dest_kernel(const u64* __restrict__ hi, u64 n, const u64* __restrict__ split, u32 nsplit,
                               u32* __restrict__ dest) {
  __shared__ u64 s[256];
  for (u32 k = threadIdx.x; k < nsplit; k += blockDim.x) s[k] = split[k];
  __syncthreads();
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const u64 h = hi[i];
    u32 a = 0, b = nsplit;  // upper bound: first splitter > h
    while (a < b) {
      const u32 m = (a + b) >> 1;
      if (s[m] <= h) a = m + 1;
      else b = m;
    }
    dest[i] = a;
  }
}

__global__ void ts_gather_kernel(const u32* __restrict__ in, const u32* __restrict__ perm, u64 n,
                                 u32* __restrict__ out) {
  const u64 nw = n * WORDS;
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 w = (u64)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += stride) {
    const u64 r = w / WORDS;
    const u32 j = (u32)(w - r * WORDS);
    out[w] = __builtin_nontemporal_load(in + clamp_row(perm[r], n) * WORDS + j);
  }
}

// v2: the same dword mapping, UNROLL independent elements per thread per
// step — all permutation loads, then all record loads, then all stores — so a
// wave has UNROLL loads in flight instead of a perm -> data -> store chain
template <int UNROLL>
__global__ void __launch_bounds__(256) ts_gather_unrolled_kernel(const u32* __restrict__ in,
                                                                 const u32* __restrict__ perm, u64 n,
                                                                 u32* __restrict__ out) {
  const u64 nw = n * WORDS;
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 w0 = (u64)blockIdx.x * blockDim.x + threadIdx.x; w0 < nw; w0 += stride * UNROLL) {
    u32 src[UNROLL];
    u32 v[UNROLL];
#pragma unroll
    for (int k = 0; k < UNROLL; ++k) {
      const u64 w = w0 + (u64)k * stride;
      const u64 r = w / WORDS;
      src[k] = w < nw ? (u32)clamp_row(perm[r], n) : 0u;
    }
#pragma unroll
    for (int k = 0; k < UNROLL; ++k) {
      const u64 w = w0 + (u64)k * stride;
      const u64 r = w / WORDS;
      const u32 j = (u32)(w - r * WORDS);
      v[k] = w < nw ? __builtin_nontemporal_load(in + (u64)src[k] * WORDS + j) : 0u;
    }
#pragma unroll
    for (int k = 0; k < UNROLL; ++k) {
      const u64 w = w0 + (u64)k * stride;
      if (w < nw) __builtin_nontemporal_store(v[k], out + w);
    }
  }
}

// v3: one record per thread: 25 independent dword loads, 25 stores
__global__ void __launch_bounds__(256) ts_gather_rec_kernel(const u32* __restrict__ in, const u32* __restrict__ perm,
                                                            u64 n, u32* __restrict__ out) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += stride) {
    const u32* p = in + clamp_row(perm[r], n) * WORDS;
    u32 v[WORDS];
#pragma unroll
    for (int j = 0; j < WORDS; ++j) v[j] = __builtin_nontemporal_load(p + j);
    u32* o = out + r * WORDS;
#pragma unroll
    for (int j = 0; j < WORDS; ++j) o[j] = v[j];
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

// Rows sorted by hi only: order each run of equal hi by lo (insertion sort of
// the permutation; stable because the LSD pass left ties in input order).
// Random 64-bit prefixes almost never tie, so this replaces 2 radix passes +
// a key gather.  Runs longer than 64 set *bad (caller falls back).
// Rows of equal (shi >> top_shift) — the bits the radix sort looked at — are
// ordered by the rest of the key, (shi, lo), with an insertion sort per run
// (one thread per run; runs longer than 64 set bad[0]: the caller then sorts
// the full key).  top_shift = 0: runs of equal hi ordered by lo; 32: the sort
// visited only the top 32 bits of hi (uniform TeraGen keys: ~2% of the rows
// sit in a run, almost all of length 2).
__global__ void ts_tie_fixup_kernel(u64* __restrict__ shi, u32* __restrict__ perm, const u64* __restrict__ lo,
                                    u64 n, u32* __restrict__ bad, int top_shift) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i + 1 < n; i += stride) {
    const u64 h = shi[i] >> top_shift;
    if ((shi[i + 1] >> top_shift) != h || (i > 0 && (shi[i - 1] >> top_shift) == h)) continue;
    u64 e = i + 2;
    while (e < n && (shi[e] >> top_shift) == h && e - i <= 64) ++e;
    if (e - i > 64) {
      atomicOr(bad, 1u);
      continue;
    }
    for (u64 a = i + 1; a < e; ++a) {
      const u32 p = perm[a];
      const u64 kh = shi[a], kl = lo[clamp_row(p, n)];
      u64 b = a;
      while (b > i) {
        const u64 ph = shi[b - 1];
        if (ph < kh || (ph == kh && lo[clamp_row(perm[b - 1], n)] <= kl)) break;
        perm[b] = perm[b - 1];
        shi[b] = ph;
        --b;
      }
      perm[b] = p;
      shi[b] = kh;
    }
  }
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

int mr_ts_dest(const void* hi, u64 n, const void* split, u32 nsplit, void* dest, hipStream_t s) {
  if (n == 0) return 0;
  if (nsplit > 256) return -1;
  hipLaunchKernelGGL(ts::ts_dest_kernel, dim3(ts_grid(n)), dim3(256), 0, s, (const u64*)hi, n, (const u64*)split,
                     nsplit, (u32*)dest);
  return (int)hipGetLastError();
}

int mr_ts_gather_mode(const void* in, const void* perm, u64 n, void* out, int mode, int grid, hipStream_t s);

// Row gather: 8 independent elements per thread per step, 16384 workgroups
// (tools/ts_gather_probe.py at 100 M records: 8.05 -> 6.58 ms; ~5 TB/s of HBM
// traffic counting the 1.77 128-byte lines a random 100-byte record touches).
int mr_ts_gather(const void* in, const void* perm, u64 n, void* out, hipStream_t s) {
  if (n == 0) return 0;
  return mr_ts_gather_mode(in, perm, n, out, 2, (int)ts_grid(n * ts::WORDS, 16384), s);
}

// mode 0: dword per thread (ts_gather_kernel); 1/2/3: UNROLL 4/8/16; 4: record per thread
int mr_ts_gather_mode(const void* in, const void* perm, u64 n, void* out, int mode, int grid, hipStream_t s) {
  if (n == 0) return 0;
  const u32* I = (const u32*)in;
  const u32* P = (const u32*)perm;
  u32* O = (u32*)out;
  const unsigned g = grid > 0 ? (unsigned)grid : ts_grid(n * ts::WORDS);
  switch (mode) {
    case 0: hipLaunchKernelGGL(ts::ts_gather_kernel, dim3(g), dim3(256), 0, s, I, P, n, O); break;
    case 1: hipLaunchKernelGGL(ts::ts_gather_unrolled_kernel<4>, dim3(g), dim3(256), 0, s, I, P, n, O); break;
    case 2: hipLaunchKernelGGL(ts::ts_gather_unrolled_kernel<8>, dim3(g), dim3(256), 0, s, I, P, n, O); break;
    case 3: hipLaunchKernelGGL(ts::ts_gather_unrolled_kernel<16>, dim3(g), dim3(256), 0, s, I, P, n, O); break;
    case 4: hipLaunchKernelGGL(ts::ts_gather_rec_kernel, dim3(grid > 0 ? (unsigned)grid : ts_grid(n)), dim3(256), 0,
                               s, I, P, n, O); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

int mr_ts_tie_fixup2(void* shi, void* perm, const void* lo, u64 n, void* bad, int top_shift, hipStream_t s) {
  if (n < 2) return 0;
  hipLaunchKernelGGL(ts::ts_tie_fixup_kernel, dim3(ts_grid(n)), dim3(256), 0, s, (u64*)shi, (u32*)perm,
                     (const u64*)lo, n, (u32*)bad, top_shift);
  return (int)hipGetLastError();
}

int mr_ts_tie_fixup(const void* shi, void* perm, const void* lo, u64 n, void* bad, hipStream_t s) {
  return mr_ts_tie_fixup2(const_cast<void*>(shi), perm, lo, n, bad, 0, s);
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
