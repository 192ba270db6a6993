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

// One thread's 16 bytes (bytes past n read as whitespace, not c): item mask
// (bit i: an item starts at byte g + i; mode 0: token start, mode 1: byte ==
// c), whitespace mask and newline mask.
struct SegMasks {
  u32 item, ws, nl;
};

__device__ __forceinline__ SegMasks seg_masks(const u8* __restrict__ text, u64 n, u64 g, int mode, u32 c) {
  u32 w[4] = {0x20202020u, 0x20202020u, 0x20202020u, 0x20202020u};
  if (g + SEG <= n && (((uintptr_t)(text + g)) & 15) == 0) {
    const uint4 q = *reinterpret_cast<const uint4*>(text + g);
    w[0] = q.x;
    w[1] = q.y;
    w[2] = q.z;
    w[3] = q.w;
  } else {
#pragma unroll
    for (int i = 0; i < SEG; ++i)
      if (g + i < n) w[i >> 2] = (w[i >> 2] & ~(0xFFu << (8 * (i & 3)))) | ((u32)text[g + i] << (8 * (i & 3)));
  }
  SegMasks r{0u, 0u, 0u};
#pragma unroll
  for (int i = 0; i < SEG; ++i) {
    const u32 b = (w[i >> 2] >> (8 * (i & 3))) & 0xFFu;
    const bool in = g + i < n;
    r.ws |= (is_ws(b) ? 1u : 0u) << i;
    r.nl |= (b == 10u && in ? 1u : 0u) << i;
    if (mode == 1) r.item |= (b == c && in ? 1u : 0u) << i;
  }
  if (mode == 0) {
    const u32 prev_ws = (g == 0 || is_ws(text[g - 1])) ? 1u : 0u;
    r.item = (~r.ws) & ((r.ws << 1) | prev_ws) & 0xFFFFu;
  }
  return r;
}

// Per tile: the number of items, and (line_counts != null) of newlines.
__global__ void __launch_bounds__(T) text_count_kernel(const u8* __restrict__ text, u64 n, int mode, u32 c,
                                                      long long* __restrict__ tile_counts,
                                                      long long* __restrict__ line_counts) {
  __shared__ u32 wsum[T / 64], nsum[T / 64];
  const u64 g = (u64)blockIdx.x * TILE + (u64)threadIdx.x * SEG;
  u32 cnt = 0, nlc = 0;
  if (g < n) {
    const SegMasks m = seg_masks(text, n, g, mode, c);
    cnt = (u32)__builtin_popcount(m.item);
    nlc = (u32)__builtin_popcount(m.nl);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    cnt += __shfl_xor(cnt, o);
    nlc += __shfl_xor(nlc, o);
  }
  if ((threadIdx.x & 63) == 0) {
    wsum[threadIdx.x >> 6] = cnt;
    nsum[threadIdx.x >> 6] = nlc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    u32 s = 0, q = 0;
#pragma unroll
    for (int w = 0; w < T / 64; ++w) {
      s += wsum[w];
      q += nsum[w];
    }
    tile_counts[blockIdx.x] = (long long)s;
    if (line_counts) line_counts[blockIdx.x] = (long long)q;
  }
}

// First position in [from, to) whose bit is set (want = 1) or clear (want =
// 0) in a tile bit mask (u32 words, bit i of word w = byte 32 w + i), or `to`.
template <int WANT>
__device__ __forceinline__ u32 tile_next_bit(const u32* w, u32 from, u32 to) {
  u32 i = from;
  while (i < to) {
    const u32 word = WANT ? w[i >> 5] : ~w[i >> 5];
    const u32 m = word >> (i & 31);
    if (m) {
      const u32 p = i + (u32)__builtin_ctz(m);
      return p < to ? p : to;
    }
    i = (i | 31) + 1;
  }
  return to;
}

// End (exclusive, global) of the n-gram whose first token ends at global
// position e: grams - 1 more tokens on the same line, each after a run of
// whitespace that holds no newline; -1 when the line ends first.  Bytes of
// the tile [tile, tile + TILE) are read from its LDS masks, later bytes from
// global memory.
__device__ __forceinline__ long long ngram_end(const u8* __restrict__ text, u64 n, u64 tile, const u32* wsw,
                                               const u32* nlw, u64 e, int grams) {
  for (int g = 1; g < grams; ++g) {
    // the next token's start: skip whitespace, but not a newline
    u64 q = e;
    if (q < tile + TILE) {
      const u32 r = tile_next_bit<0>(wsw, (u32)(q - tile), (u32)TILE);
      const u32 nl = tile_next_bit<1>(nlw, (u32)(q - tile), r);
      if (nl < r) return -1;
      q = tile + r;
    }
    if (q >= tile + TILE) {
      while (q < n && is_ws(text[q])) {
        if (text[q] == 10) return -1;
        ++q;
      }
    }
    if (q >= n) return -1;
    // its end
    u64 f = q;
    if (f < tile + TILE) f = tile + tile_next_bit<1>(wsw, (u32)(f - tile), (u32)TILE);
    if (f >= tile + TILE)
      while (f < n && !is_ws(text[f])) ++f;
    e = f;
  }
  return (long long)e;
}

// Items of a tile in text order at tile_off[tile] + rank: positions, token
// lengths (out_len) and 0-based line numbers (out_line, from the newline
// counts' exclusive scan line_off).  Token ends come from the tile's
// whitespace masks in LDS (a token past the tile continues through global
// memory); a tile's items are ranked by a wave64 scan and staged in LDS, then
// written out coalesced.
constexpr int TE_MAX = (int)TILE / 2 + 1;  // items per tile: tokens are >= 1 byte apart

__global__ void __launch_bounds__(T) text_emit_kernel(const u8* __restrict__ text, u64 n, int mode, u32 c,
                                                     const long long* __restrict__ tile_off, u64 cap,
                                                     long long* __restrict__ out_pos, int* __restrict__ out_len,
                                                     const long long* __restrict__ line_off,
                                                     long long* __restrict__ out_line) {
  __shared__ __attribute__((aligned(4))) u16 wsm[T + 2];
  __shared__ __attribute__((aligned(4))) u16 nlm[T];   // newline masks (n-grams stop at line ends)
  __shared__ u16 ipos[TILE];        // tile offsets of the items (mode 1 may have TILE of them)
  __shared__ u32 ilen[TE_MAX];      // token lengths (mode 0)
  __shared__ u16 iline[TILE];       // newlines of the tile before each item
  __shared__ u32 wsum[T / 64], nsum[T / 64];
  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  const u64 tile = (u64)blockIdx.x * TILE;
  const u64 g = tile + (u64)t * SEG;
  SegMasks m{0u, 0u, 0u};
  if (g < n) m = seg_masks(text, n, g, mode, c);
  else m.ws = 0xFFFFu;
  wsm[t] = (u16)m.ws;
  nlm[t] = (u16)m.nl;
  if (t == 0) wsm[T] = wsm[T + 1] = 0;
  const u32 cnt = (u32)__builtin_popcount(m.item);
  const u32 nlc = (u32)__builtin_popcount(m.nl);
  u32 ci = cnt, ni = nlc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const u32 a = __shfl_up(ci, o), b = __shfl_up(ni, o);
    if (lane >= o) {
      ci += a;
      ni += b;
    }
  }
  if (lane == 63) {
    wsum[wave] = ci;
    nsum[wave] = ni;
  }
  __syncthreads();
  u32 cb = 0, nb = 0, total = 0;
#pragma unroll
  for (int w = 0; w < T / 64; ++w) {
    cb += w < wave ? wsum[w] : 0u;
    nb += w < wave ? nsum[w] : 0u;
    total += wsum[w];
  }
  u32 k = cb + ci - cnt;         // this thread's first item rank in the tile
  const u32 nl0 = nb + ni - nlc;  // newlines of the tile before this segment
  u32 it = m.item;
  while (it) {
    const int i = __builtin_ctz(it);
    it &= it - 1;
    ipos[k] = (u16)(t * SEG + i);
    if (out_line) iline[k] = (u16)(nl0 + (u32)__builtin_popcount(m.nl & ((1u << i) - 1u)));
    if (out_len) {
      // the token's end: the next whitespace byte (own mask, then the next
      // segments' masks in LDS, then global memory past the tile)
      u32 rest = (m.ws >> (i + 1)) << (i + 1);
      u32 e;
      if (rest) {
        e = t * SEG + (u32)__builtin_ctz(rest);
      } else {
        int s2 = t + 1;
        e = (u32)TILE;
        for (; s2 < T; ++s2) {
          const u32 w2 = wsm[s2];
          if (w2) {
            e = (u32)s2 * SEG + (u32)__builtin_ctz(w2);
            break;
          }
        }
      }
      u64 ge = tile + e;
      if (e == (u32)TILE)
        while (ge < n && !is_ws(text[ge])) ++ge;
      const u64 gs = tile + t * SEG + i;
      if (c >= 2) {  // n-gram spans (c tokens of one line) instead of token lengths; 0: none
        const long long ne = ngram_end(text, n, tile, (const u32*)wsm, (const u32*)nlm, ge, (int)c);
        ilen[k] = ne < 0 ? 0u : (u32)((u64)ne - gs);
      } else {
        ilen[k] = (u32)(ge - gs);
      }
    }
    ++k;
  }
  __syncthreads();
  const u64 k0 = (u64)tile_off[blockIdx.x];
  const long long lb = out_line ? line_off[blockIdx.x] : 0;
  for (u32 x = t; x < total; x += T) {
    const u64 q = k0 + x;
    if (q >= cap) break;
    out_pos[q] = (long long)(tile + ipos[x]);
    if (out_len) out_len[q] = (int)ilen[x];
    if (out_line) out_line[q] = lb + (long long)iline[x];
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

// line_counts (optional): per-tile newline counts (for mr_text_emit's line numbers)
int mr_text_count(const void* text, u64 n, int mode, u32 c, void* tile_counts, void* line_counts, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(text_count_kernel, dim3((unsigned)mr_text_tiles(n)), dim3(T), 0, s, (const u8*)text, n, mode, c,
                     (long long*)tile_counts, (long long*)line_counts);
  return (int)hipGetLastError();
}

// out_len (mode 0) and out_line (with line_off = exclusive scan of the newline
// counts) are optional.
// mode 0 with c >= 2: out_len = the span of the c-token n-gram starting at each
// token (0: fewer than c tokens left on its line) instead of its length.
int mr_text_emit(const void* text, u64 n, int mode, u32 c, const void* tile_off, u64 cap, void* out_pos,
                 void* out_len, const void* line_off, void* out_line, hipStream_t s) {
  if (n == 0) return 0;
  if (out_len && mode != 0) return -1;
  if (mode == 0 && c > 64) return -1;
  if (out_line && !line_off) return -1;
  hipLaunchKernelGGL(text_emit_kernel, dim3((unsigned)mr_text_tiles(n)), dim3(T), 0, s, (const u8*)text, n, mode, c,
                     (const long long*)tile_off, cap, (long long*)out_pos, (int*)out_len,
                     (const long long*)line_off, (long long*)out_line);
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
