// text.hip — ordered text scanning and field parsing for user device map
// functions (ops/text.py): the building blocks a device_mapfn uses to pick
// its keys and values out of the staged input bytes, in place of the
// reference's Lua string functions (``line:gmatch("[^%s]+")``,
// examples/WordCount/mapfn.lua:5; ``io.lines``, mapfn.lua:4; ``tonumber``).
//
//   text_count / text_emit : positions, in text order, of every token start
//       (maximal run of non-%s bytes, with its length) or of every byte equal
//       to a given one (newlines, separators).  Two passes over 4 KiB tiles:
//       per-tile counts -> exclusive scan (sort.hip) -> each thread writes its
//       items at tile offset + block-scan rank, so the output is ordered.
//   text_field            : byte span of field k of each line (sep-separated).
//   text_parse_f64 / _i64 : decimal numbers of byte spans.
#include <hip/hip_runtime.h>
#include "mr_common.h"
#include "text_parse.h"

namespace mr {
namespace tx {

constexpr int T = 256;
constexpr int SEG = 16;
constexpr u64 TILE = (u64)T * SEG;  // 4096 bytes per workgroup

// Bit i of the result: an item starts at byte g + i (mode 0: token start,
// mode 1: byte == c).  Bytes past n are whitespace / not c.
__device__ __forceinline__ u32 item_mask(const u8* __restrict__ text, u64 n, u64 g, int mode, u32 c) {
  u32 b[SEG];
  if (g + SEG <= n && (((uintptr_t)(text + g)) & 15) == 0) {
    const uint4 q = *reinterpret_cast<const uint4*>(text + g);
    const u32 w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < SEG; ++i) b[i] = (w[i >> 2] >> (8 * (i & 3))) & 0xFFu;
  } else {
#pragma unroll
    for (int i = 0; i < SEG; ++i) b[i] = g + i < n ? (u32)text[g + i] : 32u;
  }
  u32 m = 0;
  if (mode == 1) {
#pragma unroll
    for (int i = 0; i < SEG; ++i) m |= (b[i] == c && g + i < n ? 1u : 0u) << i;
    return m;
  }
  u32 ws = 0;
#pragma unroll
  for (int i = 0; i < SEG; ++i) ws |= (is_ws(b[i]) ? 1u : 0u) << i;
  const u32 prev_ws = (g == 0 || is_ws(text[g - 1])) ? 1u : 0u;
  return (~ws) & ((ws << 1) | prev_ws) & 0xFFFFu;
}

__global__ void __launch_bounds__(T) text_count_kernel(const u8* __restrict__ text, u64 n, int mode, u32 c,
                                                      long long* __restrict__ tile_counts) {
  __shared__ u32 wsum[T / 64];
  const u64 g = (u64)blockIdx.x * TILE + (u64)threadIdx.x * SEG;
  u32 cnt = g < n ? (u32)__builtin_popcount(item_mask(text, n, g, mode, c)) : 0u;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    u32 s = 0;
#pragma unroll
    for (int w = 0; w < T / 64; ++w) s += wsum[w];
    tile_counts[blockIdx.x] = (long long)s;
  }
}

__global__ void __launch_bounds__(T) text_emit_kernel(const u8* __restrict__ text, u64 n, int mode, u32 c,
                                                     const long long* __restrict__ tile_off, u64 cap,
                                                     long long* __restrict__ out_pos, int* __restrict__ out_len) {
  __shared__ u32 sh[T];
  const int t = threadIdx.x;
  const u64 g = (u64)blockIdx.x * TILE + (u64)t * SEG;
  u32 m = g < n ? item_mask(text, n, g, mode, c) : 0u;
  const u32 cnt = (u32)__builtin_popcount(m);
  sh[t] = cnt;
  __syncthreads();
  for (int o = 1; o < T; o <<= 1) {
    const u32 y = t >= o ? sh[t - o] : 0u;
    __syncthreads();
    sh[t] += y;
    __syncthreads();
  }
  u64 k = (u64)tile_off[blockIdx.x] + sh[t] - cnt;
  while (m) {
    const int i = __builtin_ctz(m);
    m &= m - 1;
    const u64 p = g + i;
    if (k < cap) {
      out_pos[k] = (long long)p;
      if (out_len) {
        u64 e = p + 1;
        while (e < n && !is_ws(text[e])) ++e;
        out_len[k] = (int)(e - p);
      }
    }
    ++k;
  }
}

// Span of field k (0-based) of each line: bytes between the k-th and (k+1)-th
// separator (or the line's ends).  A trailing '\r' of the line is not part of
// its last field.  Missing field: start -1, length 0.
__global__ void text_field_kernel(const u8* __restrict__ text, const long long* __restrict__ ls,
                                  const int* __restrict__ ll, u64 m, u32 sep, int k, long long* __restrict__ fs,
                                  int* __restrict__ fl) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) {
    const long long s = ls[i];
    int len = ll[i];
    if (len > 0 && text[s + len - 1] == '\r') --len;
    int f = 0, a = 0;
    int j = 0;
    for (; j < len && f < k; ++j)
      if (text[s + j] == sep) {
        ++f;
        a = j + 1;
      }
    if (f < k || len <= 0) {
      fs[i] = -1;
      fl[i] = 0;
      continue;
    }
    int e = a;
    while (e < len && text[s + e] != sep) ++e;
    fs[i] = s + a;
    fl[i] = e - a;
  }
}

__global__ void text_parse_f64_kernel(const u8* __restrict__ text, const long long* __restrict__ s,
                                      const int* __restrict__ l, u64 m, double* __restrict__ out,
                                      unsigned int* __restrict__ err) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  bool anybad = false;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) {
    bool bad = s[i] < 0;
    const double v = bad ? 0.0 : parse_f64(text + s[i], l[i], bad);
    out[i] = bad ? __longlong_as_double(0x7FF8000000000000ll) : v;
    anybad |= bad;
  }
  if (anybad && err) atomicOr(err, 1u);
}

__global__ void text_parse_i64_kernel(const u8* __restrict__ text, const long long* __restrict__ s,
                                      const int* __restrict__ l, u64 m, long long* __restrict__ out,
                                      unsigned int* __restrict__ err) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  bool anybad = false;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) {
    long long v = 0;
    bool bad = s[i] < 0;
    if (!bad) {
      const u8* p = text + s[i];
      const int len = l[i];
      int j = 0;
      while (j < len && is_ws(p[j])) ++j;
      bool neg = false;
      if (j < len && (p[j] == '+' || p[j] == '-')) neg = p[j++] == '-';
      u64 a = 0;
      int nd = 0;
      for (; j < len && p[j] >= '0' && p[j] <= '9'; ++j, ++nd) a = a * 10 + (p[j] - '0');
      while (j < len && is_ws(p[j])) ++j;
      bad = nd == 0 || j != len || nd > 19;
      v = neg ? -(long long)a : (long long)a;
    }
    out[i] = bad ? 0 : v;
    anybad |= bad;
  }
  if (anybad && err) atomicOr(err, 1u);
}

}  // namespace tx
}  // namespace mr

using namespace mr;
using namespace mr::tx;

static inline unsigned tx_grid(u64 n, unsigned block, unsigned cap = 8192) {
  u64 g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

extern "C" {

u64 mr_text_tiles(u64 n) { return (n + TILE - 1) / TILE; }

int mr_text_count(const void* text, u64 n, int mode, u32 c, void* tile_counts, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(text_count_kernel, dim3((unsigned)mr_text_tiles(n)), dim3(T), 0, s, (const u8*)text, n, mode, c,
                     (long long*)tile_counts);
  return (int)hipGetLastError();
}

int mr_text_emit(const void* text, u64 n, int mode, u32 c, const void* tile_off, u64 cap, void* out_pos,
                 void* out_len, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(text_emit_kernel, dim3((unsigned)mr_text_tiles(n)), dim3(T), 0, s, (const u8*)text, n, mode, c,
                     (const long long*)tile_off, cap, (long long*)out_pos, (int*)out_len);
  return (int)hipGetLastError();
}

int mr_text_field(const void* text, const void* ls, const void* ll, u64 m, u32 sep, int k, void* fs, void* fl,
                  hipStream_t s) {
  if (m == 0) return 0;
  hipLaunchKernelGGL(text_field_kernel, dim3(tx_grid(m, 256)), dim3(256), 0, s, (const u8*)text,
                     (const long long*)ls, (const int*)ll, m, sep, k, (long long*)fs, (int*)fl);
  return (int)hipGetLastError();
}

int mr_text_parse_f64(const void* text, const void* st, const void* ln, u64 m, void* out, void* err, hipStream_t s) {
  if (m == 0) return 0;
  hipLaunchKernelGGL(text_parse_f64_kernel, dim3(tx_grid(m, 256)), dim3(256), 0, s, (const u8*)text,
                     (const long long*)st, (const int*)ln, m, (double*)out, (unsigned int*)err);
  return (int)hipGetLastError();
}

int mr_text_parse_i64(const void* text, const void* st, const void* ln, u64 m, void* out, void* err, hipStream_t s) {
  if (m == 0) return 0;
  hipLaunchKernelGGL(text_parse_i64_kernel, dim3(tx_grid(m, 256)), dim3(256), 0, s, (const u8*)text,
                     (const long long*)st, (const int*)ln, m, (long long*)out, (unsigned int*)err);
  return (int)hipGetLastError();
}

}  // extern "C"
