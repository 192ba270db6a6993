// records.hip — the record plane's kernels for rows of any width (gfx950):
// fixed-width records moved, not folded (device_reduce = "identity";
// parallel/planes.py RecordPlane), keyed by their first `kb` bytes (kb <= 16,
// unsigned bytewise order = the reference's string key order, utils.lua:126).
// TeraSort's 100-byte rows with 10-byte keys are one shape of it.
//
// The sort is a 32-bit radix sort of the key prefixes plus an exact fix-up:
//   rec_keys32   : k32 = key bytes 0..3 big-endian, and the radix sort's digit
//                  histograms of k32 in the same pass (no histogram pass);
//   (sort.hip)   : 4 onesweep passes over (k32, u32 row) — u32 keys: 16 bytes
//                  moved per row and pass instead of 24 with u64 keys;
//   rec_tie_*    : rows equal in k32 ordered by key bytes 4..kb-1 read from the
//                  rows themselves (uniform keys: ~2 % of the rows sit in such
//                  a run, almost all of length 2): a streaming scan lists each
//                  block's run starts, one thread per listed pair swaps it,
//                  longer runs are insertion-sorted by a third kernel; a run
//                  longer than 64 (or a block with too many runs) sets *bad and
//                  the caller sorts the full (hi, lo) key instead;
//   rec_gather16 : output row i = input row perm[i] with 16-byte loads and
//                  stores through LDS (rows of 16-244 bytes, a multiple of 4);
//                  rec_gather (one word per lane) and rec_gather_bytes for the
//                  other widths.  The random row reads touch 1.75 128-byte
//                  lines per 100-byte row: the gather runs near the HBM rate
//                  on those lines.
//   rec_keys     : full (hi, lo) key words (fallback sort, sampling, checks);
//   rec_dest32   : range partition = number of splitters <= k32.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "mr_common.h"

namespace mr {
namespace rc {

// Big-endian u32 of bytes [b, b+4) of a row, bytes at or past kb read as 0.
__device__ __forceinline__ u32 be32(const u8* row, int b, int kb, bool words) {
  if (words && b + 4 <= kb) return __builtin_bswap32(*reinterpret_cast<const u32*>(row + b));
  u32 v = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) v = (v << 8) | (b + j < kb ? (u32)row[b + j] : 0u);
  return v;
}

__device__ __forceinline__ u64 be64(const u8* row, int b, int kb, bool words) {
  return ((u64)be32(row, b, kb, words) << 32) | (u64)be32(row, b + 4, kb, words);
}

// k32 of every row (+ digit histograms of k32 into ghist[0..3][256] when
// ghist is given: zeroed u32 [8][256]).  256 threads, grid-stride.
__global__ void __launch_bounds__(256) rec_keys32_kernel(const u8* __restrict__ rec, u64 n, int rb, int kb,
                                                         u32* __restrict__ k32, u32* __restrict__ ghist) {
  __shared__ u32 h[4][256];
  const int t = threadIdx.x;
  if (ghist) {
#pragma unroll
    for (int b = 0; b < 4; ++b) h[b][t] = 0;
    __syncthreads();
  }
  const bool words = (rb & 3) == 0;
  const u64 stride = (u64)gridDim.x * blockDim.x;
  // one 4-byte load per 100-byte row: the pass reads every line of the rows
  // (2.0 ms per 10 GB, ~5 TB/s; 8 loads in flight per thread measured no
  // faster, profiles/r3/check7/ts_ab_box2.log)
  for (u64 i = (u64)blockIdx.x * blockDim.x + t; i < n; i += stride) {
    const u32 k = be32(rec + i * (u64)rb, 0, kb, words);
    k32[i] = k;
    if (ghist) {
#pragma unroll
      for (int b = 0; b < 4; ++b) atomicAdd(&h[b][(k >> (8 * b)) & 0xFFu], 1u);
    }
  }
  if (ghist) {
    __syncthreads();
#pragma unroll
    for (int b = 0; b < 4; ++b)
      if (h[b][t]) atomicAdd(&ghist[b * 256 + t], h[b][t]);
  }
}

__global__ void rec_keys_kernel(const u8* __restrict__ rec, u64 n, int rb, int kb, u64* __restrict__ hi,
                                u64* __restrict__ lo) {
  const bool words = (rb & 3) == 0;
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const u8* row = rec + i * (u64)rb;
    hi[i] = be64(row, 0, kb, words);
    lo[i] = be64(row, 8, kb, words);
  }
}

// The rest of a key after its 32-bit prefix: bytes 4..15 as (u64, u32).
__device__ __forceinline__ void key_rest(const u8* row, int kb, bool words, u64& a, u32& b) {
  a = be64(row, 4, kb, words);
  b = be32(row, 12, kb, words);
}

// Runs of equal k32 in the sorted prefixes, ordered by the rest of their keys
// (bytes 4..kb-1 read from the rows; stable: the LSD sort left equal keys in
// input order).  Uniform keys: ~2 % of the rows sit in a run, almost all of
// length 2 — rec_tie_fix_kernel swaps those and appends the start of every
// longer run to a list; rec_tie_runs_kernel sorts the listed runs (insertion
// sort, one thread per run).  A run longer than 64 sets *bad and the caller
// sorts the full (hi, lo) key instead.
constexpr int TIE_MAX = 64;

// Two streaming-friendly steps (a single kernel that swapped pairs where it
// found them waited on a dependent perm -> row load chain in every wave that
// held a pair: 0.56 ms per 100 M rows against 0.24): rec_tie_scan_kernel only reads the sorted
// prefixes and keeps each block's run starts (TS_POS positions per block, at
// most TS_CAP starts, in LDS, then in the block's own segment — no global
// atomics); rec_tie_fix_kernel then gives every listed run a thread of its
// own, so all the random loads are independent.  Runs of 3 or more go to the
// run list of rec_tie_runs_kernel as before.
constexpr int TS_POS = 4096;
constexpr int TS_CAP = 1024;

__global__ void __launch_bounds__(256) rec_tie_scan_kernel(const u32* __restrict__ sk, u64 n,
                                                           u32* __restrict__ counts, u32* __restrict__ seg,
                                                           u32* __restrict__ bad) {
  __shared__ u32 cnt;
  __shared__ u32 list[TS_CAP];
  const u32 t = threadIdx.x;
  if (t == 0) cnt = 0;
  __syncthreads();
  const u64 base = (u64)blockIdx.x * TS_POS;
  const bool al = (((uintptr_t)sk & 15) == 0);
#pragma unroll
  for (int it = 0; it < TS_POS / 1024; ++it) {
    const u64 i0 = base + (u64)it * 1024 + 4ull * t;
    if (i0 >= n) break;
    u32 v[7];  // sk[i0 - 1 .. i0 + 5]
    if (i0 + 4 <= n && al) {
      const uint4 q = *reinterpret_cast<const uint4*>(sk + i0);
      v[1] = q.x; v[2] = q.y; v[3] = q.z; v[4] = q.w;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[1 + j] = i0 + j < n ? sk[i0 + j] : 0u;
    }
    v[0] = i0 > 0 ? sk[i0 - 1] : ~v[1];
    v[5] = i0 + 4 < n ? sk[i0 + 4] : 0u;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const u64 i = i0 + j;
      if (i + 1 >= n) break;
      const u32 h = v[1 + j];
      if (v[2 + j] == h && v[j] != h) {  // the start of a run
        const u32 k = atomicAdd(&cnt, 1u);
        if (k < (u32)TS_CAP) list[k] = (u32)(i - base);
      }
    }
  }
  __syncthreads();
  const u32 m = cnt;
  const u32 keep = m < (u32)TS_CAP ? m : (u32)TS_CAP;
  if (t == 0) {
    counts[blockIdx.x] = keep;
    if (m > (u32)TS_CAP) atomicOr(bad, 1u);  // > 1/4 of the rows start a tie run: full-key sort
  }
  for (u32 k = t; k < keep; k += 256) seg[(u64)blockIdx.x * TS_CAP + k] = list[k];
}

__global__ void __launch_bounds__(256) rec_tie_fix_kernel(const u32* __restrict__ sk, u32* __restrict__ perm,
                                                          const u8* __restrict__ rec, u64 n, int rb, int kb,
                                                          const u32* __restrict__ counts,
                                                          const u32* __restrict__ seg, u32* __restrict__ bad,
                                                          u64* __restrict__ runs,
                                                          unsigned long long* __restrict__ nruns, u64 runs_cap) {
  const bool words = (rb & 3) == 0;
  const u32 m = counts[blockIdx.x];
  const u64 base = (u64)blockIdx.x * TS_POS;
  for (u32 k = threadIdx.x; k < m; k += 256) {
    const u64 i = base + seg[(u64)blockIdx.x * TS_CAP + k];
    if (i + 1 >= n) continue;
    const u32 h = sk[i];
    if (i + 2 < n && sk[i + 2] == h) {  // a run of 3 or more
      const unsigned long long x = atomicAdd(nruns, 1ull);
      if (x < runs_cap) runs[x] = i;
      else atomicOr(bad, 1u);
      continue;
    }
    const u32 p0 = perm[i], p1 = perm[i + 1];
    u64 a0, a1;
    u32 b0, b1;
    key_rest(rec + (u64)clamp_row(p0, n) * rb, kb, words, a0, b0);
    key_rest(rec + (u64)clamp_row(p1, n) * rb, kb, words, a1, b1);
    if (a0 > a1 || (a0 == a1 && b0 > b1)) {
      perm[i] = p1;
      perm[i + 1] = p0;
    }
  }
}

__global__ void __launch_bounds__(64) rec_tie_runs_kernel(const u32* __restrict__ sk, u32* __restrict__ perm,
                                                          const u8* __restrict__ rec, u64 n, int rb, int kb,
                                                          u32* __restrict__ bad, const u64* __restrict__ runs,
                                                          const unsigned long long* __restrict__ nruns,
                                                          u64 runs_cap) {
  const bool words = (rb & 3) == 0;
  const u64 m_runs = min((u64)*nruns, runs_cap);
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 x = (u64)blockIdx.x * blockDim.x + threadIdx.x; x < m_runs; x += stride) {
    const u64 i = runs[x];
    const u32 h = sk[i];
    u64 e = i + 2;
    while (e < n && sk[e] == h && e - i <= TIE_MAX) ++e;
    if (e - i > TIE_MAX) {
      atomicOr(bad, 1u);
      continue;
    }
    u64 ra[TIE_MAX];
    u32 rb2[TIE_MAX];
    u32 p[TIE_MAX];
    const int m = (int)(e - i);
    for (int a = 0; a < m; ++a) {
      p[a] = perm[i + a];
      key_rest(rec + (u64)clamp_row(p[a], n) * rb, kb, words, ra[a], rb2[a]);
    }
    for (int a = 1; a < m; ++a) {
      const u64 ka = ra[a];
      const u32 kb2 = rb2[a];
      const u32 pa = p[a];
      int b = a;
      while (b > 0 && (ra[b - 1] > ka || (ra[b - 1] == ka && rb2[b - 1] > kb2))) {
        ra[b] = ra[b - 1];
        rb2[b] = rb2[b - 1];
        p[b] = p[b - 1];
        --b;
      }
      ra[b] = ka;
      rb2[b] = kb2;
      p[b] = pa;
    }
    for (int a = 0; a < m; ++a) perm[i + a] = p[a];
  }
}

// Row gather, rows of W words (W > 0: compile-time width; W == 0: `words`
// at run time), UNROLL independent words per thread: all permutation loads,
// then all row loads, then all stores (tools/ts_gather_probe.py: 8 in flight).
template <int W, int UNROLL>
__global__ void __launch_bounds__(256) rec_gather_kernel(const u32* __restrict__ in, u64 nin,
                                                         const u32* __restrict__ perm, u64 n, u32 words,
                                                         u32* __restrict__ out) {
  const u64 ww = W > 0 ? (u64)W : (u64)words;
  const u64 nw = n * ww;
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 w0 = (u64)blockIdx.x * blockDim.x + threadIdx.x; w0 < nw; w0 += stride * UNROLL) {
    u64 src[UNROLL];
    u32 v[UNROLL];
#pragma unroll
    for (int k = 0; k < UNROLL; ++k) {
      const u64 w = w0 + (u64)k * stride;
      const u64 r = w / ww;
      const u64 j = w - r * ww;
      src[k] = w < nw ? (u64)clamp_row(perm[r], nin) * ww + j : 0u;
    }
#pragma unroll
    for (int k = 0; k < UNROLL; ++k) {
      const u64 w = w0 + (u64)k * stride;
      v[k] = w < nw ? __builtin_nontemporal_load(in + src[k]) : 0u;
    }
#pragma unroll
    for (int k = 0; k < UNROLL; ++k) {
      const u64 w = w0 + (u64)k * stride;
      if (w < nw) __builtin_nontemporal_store(v[k], out + w);
    }
  }
}

// Row gather through LDS with 16-byte accesses on both sides, for rows of rb
// bytes (rb % 4 == 0, 16 <= rb <= 244; buffers 4-byte aligned: row slices
// of a larger block take the 16-byte path too, with head bytes).  A row
// starts 0/4/8/12 bytes into an aligned 16-byte chunk, so C = ceil((rb + 12) /
// 16) aligned chunks cover it whatever its position: the block loads the C
// chunks of each of its R rows (one dwordx4 per lane, all independent),
// keeps them in LDS as an image of the aligned source with each row's start
// offset, and writes its R output rows — R * rb bytes, contiguous and 16-byte
// aligned — as dwordx4 stores assembled from that image.  The dword form
// (rec_gather_kernel) issues 4x the vector-memory instructions for the same
// bytes; the windowed-permutation probe (profiles/r3/check1/ts_move.log: 8 MB
// windows no faster than random rows) says instructions, not DRAM, bound it.
template <int C, int R, bool PIPE, bool HEAD>
__global__ void __launch_bounds__(256) rec_gather16_kernel(const u8* __restrict__ in, u64 nin,
                                                           const u32* __restrict__ perm, u64 n, u32 rb,
                                                           u8* __restrict__ out, u32 ih, u32 oh) {
  typedef u32 v4u __attribute__((ext_vector_type(4)));
  __shared__ v4u img[R * C];
  __shared__ u32 mis[R];
  constexpr int PER = (R * C + 255) / 256;
  const u32 t = threadIdx.x;
  // HEAD: a buffer starts ih / oh bytes past a 16-byte boundary (row slices);
  // the aligned instantiation keeps round 5's store loop
  if constexpr (!HEAD) ih = oh = 0;
  const u64 in_bytes = nin * (u64)rb + ih;
  const u64 nbatch = (n + R - 1) / R;
  const float inv_rb = 1.0f / (float)rb;
  const u32* img32 = reinterpret_cast<const u32*>(img);
  // PIPE: the next batch's row loads are issued before this batch's stores
  // (its offsets kept in registers until the LDS image is free), so a block
  // keeps loads in flight through its store phase
  v4u v[PER];
  u32 mv[PER];
  auto load = [&](u64 bb) {
    const u64 q0 = bb * (u64)R;
    const u32 qrows = (u32)min((u64)R, n - q0);
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const u32 idx = t + 256u * k;
      const u32 row = idx / C, c = idx - row * C;
      v[k] = v4u{0u, 0u, 0u, 0u};
      mv[k] = 0xFFFFFFFFu;
      if (idx < (u32)(R * C) && row < qrows) {
        const u64 sb = (u64)clamp_row(perm[q0 + row], nin) * rb + ih;
        const u64 a = (sb & ~15ull) + 16ull * c;
        if (a + 16 <= in_bytes) {
          v[k] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(in + a));
        } else {  // the chunk that runs past the buffer's end (in_bytes % 16 != 0)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (a + 4 * j < in_bytes) v[k][j] = *reinterpret_cast<const u32*>(in + a + 4 * j);
        }
        if (c == 0) mv[k] = (u32)(sb & 15);
      }
    }
  };
  if (PIPE && (u64)blockIdx.x < nbatch) load(blockIdx.x);
  for (u64 b = blockIdx.x; b < nbatch; b += gridDim.x) {
    const u64 r0 = b * (u64)R;
    const u32 rows = (u32)min((u64)R, n - r0);
    if (!PIPE) load(b);
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const u32 idx = t + 256u * k;
      if (idx < (u32)(R * C)) img[idx] = v[k];
      if (mv[k] != 0xFFFFFFFFu) mis[idx / C] = mv[k];
    }
    __syncthreads();
    if (PIPE && b + gridDim.x < nbatch) load(b + gridDim.x);
    if constexpr (!HEAD) {
      const u32 obytes = rows * rb;  // < 2^16 for R <= 256, rb <= 244
      u8* ob = out + r0 * rb;
      const u32 nch = obytes >> 4;
      for (u32 oc = t; oc < nch + 1; oc += 256) {
        const u32 byte0 = oc * 16u;
        if (byte0 >= obytes) break;
        u32 row = (u32)((float)byte0 * inv_rb);  // exact after the corrections (byte0 < 2^24)
        if (row * rb > byte0) --row;
        if ((row + 1) * rb <= byte0) ++row;
        const u32 off = byte0 - row * rb;
        u32 w[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          u32 rr = row, oo = off + 4u * j;
          if (oo >= rb) {
            ++rr;
            oo -= rb;
          }
          w[j] = rr < rows ? img32[(rr * (u32)C * 16u + mis[rr] + oo) >> 2] : 0u;
        }
        if (oc < nch) {
          __builtin_nontemporal_store(v4u{w[0], w[1], w[2], w[3]}, reinterpret_cast<v4u*>(ob + byte0));
        } else {  // the batch's last partial chunk (rows * rb % 16 != 0): dwords
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (byte0 + 4u * j < obytes) *reinterpret_cast<u32*>(ob + byte0 + 4u * j) = w[j];
        }
      }
    } else {
      const u32 obytes = rows * rb;  // < 2^16 for R <= 256, rb <= 244
      // the batch's bytes sit oh bytes into aligned 16-byte chunks (R * rb is a
      // multiple of 16): chunks wholly inside them are dwordx4 stores, the
      // first (oh != 0) and the last partial chunk dword stores
      u8* ob = out + r0 * rb;
      const u32 nch = (obytes + oh + 15) >> 4;
      for (u32 oc = t; oc < nch; oc += 256) {
        const int b0 = (int)(oc * 16u) - (int)oh;  // batch byte of the chunk's word 0 (< 0: before the batch)
        const u32 s0 = b0 < 0 ? 0u : (u32)b0;
        u32 row = (u32)((float)s0 * inv_rb);  // exact after the corrections (s0 < 2^24)
        if (row * rb > s0) --row;
        if ((row + 1) * rb <= s0) ++row;
        const u32 off = s0 - row * rb;
        u32 w[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int lb = b0 + 4 * j;
          u32 rr = row, oo = off + (u32)(lb - (int)s0);
          if (oo >= rb) {
            ++rr;
            oo -= rb;
          }
          w[j] = lb >= 0 && rr < rows ? img32[(rr * (u32)C * 16u + mis[rr] + oo) >> 2] : 0u;
        }
        if (b0 >= 0 && (u32)b0 + 16u <= obytes) {
          __builtin_nontemporal_store(v4u{w[0], w[1], w[2], w[3]}, reinterpret_cast<v4u*>(ob + oc * 16u));
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int lb = b0 + 4 * j;
            if (lb >= 0 && (u32)lb < obytes) *reinterpret_cast<u32*>(ob + oc * 16u + 4u * j) = w[j];
          }
        }
      }
    }
    __syncthreads();
  }
}

// Rows whose width is not a multiple of 4 bytes: one byte per thread.
__global__ void rec_gather_bytes_kernel(const u8* __restrict__ in, u64 nin, const u32* __restrict__ perm, u64 n,
                                        u64 rb, u8* __restrict__ out) {
  const u64 nb = n * rb;
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 b = (u64)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += stride) {
    const u64 r = b / rb;
    out[b] = in[(u64)clamp_row(perm[r], nin) * rb + (b - r * rb)];
  }
}

__global__ void rec_dest32_kernel(const u32* __restrict__ k32, u64 n, const u32* __restrict__ split, u32 nsplit,
                                  u32* __restrict__ dest) {
  __shared__ u32 s[1024];
  for (u32 k = threadIdx.x; k < nsplit; k += blockDim.x) s[k] = split[k];
  __syncthreads();
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const u32 h = k32[i];
    u32 a = 0, b = nsplit;  // upper bound: first splitter > h
    while (a < b) {
      const u32 m = (a + b) >> 1;
      if (s[m] <= h) a = m + 1;
      else b = m;
    }
    dest[i] = a;
  }
}

// The exchange bucket of every row for the record plane's exchange pipelined
// by key range (parallel/planes.py _exchange_ranges): sub-range a = number of
// sub-splitters <= k32, partition a / K, round a % K -> bucket
// (a % K) * W + a / K, plus the buckets' histogram (= the rows per bucket, and
// digit 0 of the one-pass u32 sort that orders the rows by bucket): one pass
// instead of dest32 + four elementwise ops + an 8-bit u64 sort + bincount.
__global__ void __launch_bounds__(256) rec_bucket32_kernel(const u32* __restrict__ k32, u64 n,
                                                           const u32* __restrict__ split, u32 nsplit, u32 K, u32 W,
                                                           u32* __restrict__ bucket, u32* __restrict__ ghist) {
  __shared__ u32 s[1024];
  __shared__ u32 h[256];
  const int t = threadIdx.x;
  for (u32 k = t; k < nsplit; k += blockDim.x) s[k] = split[k];
  h[t] = 0;
  __syncthreads();
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + t; i < n; i += stride) {
    const u32 x = k32[i];
    u32 a = 0, b = nsplit;
    while (a < b) {
      const u32 m = (a + b) >> 1;
      if (s[m] <= x) a = m + 1;
      else b = m;
    }
    const u32 q = a / K;
    const u32 bk = (a - q * K) * W + q;
    bucket[i] = bk;
    atomicAdd(&h[bk], 1u);
  }
  __syncthreads();
  if (h[t]) atomicAdd(&ghist[t], h[t]);
}

// Digit histograms ([4][256], digits 0..3) of 32-bit key prefixes already
// extracted (the range-pipelined exchange ships them with the rows, so the
// receiver's sort skips its key pass over the rows).
__global__ void __launch_bounds__(256) rec_hist32_kernel(const u32* __restrict__ k32, u64 n, u32* __restrict__ ghist) {
  __shared__ u32 h[4][256];
  const int t = threadIdx.x;
#pragma unroll
  for (int b = 0; b < 4; ++b) h[b][t] = 0;
  __syncthreads();
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + t; i < n; i += stride) {
    const u32 k = k32[i];
#pragma unroll
    for (int b = 0; b < 4; ++b) atomicAdd(&h[b][(k >> (8 * b)) & 0xFFu], 1u);
  }
  __syncthreads();
#pragma unroll
  for (int b = 0; b < 4; ++b)
    if (h[b][t]) atomicAdd(&ghist[b * 256 + t], h[b][t]);
}

// Splitter sampling of the record plane (parallel/planes.py
// _sample_splitters) in three launches instead of ~20 small torch ops (the
// W = 8 step's preparation was host-bound on them, ~25 us of host time each):
// rec_sample32 draws k rows with a counter-based hash (row = fmix64(seed, j)
// mod n) and writes their 32-bit key prefixes as int64 (-1 for a rank
// without rows); after the all-gather and a sort, rec_pick takes the R - 1
// splitters at evenly spaced ranks of the non-negative entries.
__global__ void rec_sample32_kernel(const u32* __restrict__ k32, u64 n, u32 k, u64 seed, long long* __restrict__ out) {
  const u32 j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= k) return;
  out[j] = n ? (long long)k32[fmix64(seed * 0x9E3779B97F4A7C15ull + j) % n] : -1ll;
}

__global__ void rec_pick_kernel(const long long* __restrict__ srt, u64 N, u32 R, u32* __restrict__ sp) {
  // the negatives (empty ranks) sort first: the first non-negative index
  u64 a = 0, b = N;
  while (a < b) {
    const u64 m = (a + b) >> 1;
    if (srt[m] < 0) a = m + 1;
    else b = m;
  }
  const u64 m = N - a;
  for (u32 j = threadIdx.x + 1; j < R; j += blockDim.x) {
    u64 i = a + m * j / R;
    if (i >= N) i = N - 1;
    sp[j - 1] = m ? (u32)srt[i] : 0u;
  }
}

// The count-exchange rows of the range-pipelined exchange, from the bucket
// histogram: xchg[d][k] = rows for destination d in round k (bucket k*W + d),
// xchg[d][K] = this rank's failed maps; flag = the bucket sort gave up.
__global__ void rec_xchg_kernel(const u32* __restrict__ gh, u32 K, u32 W, long long failed, const u32* __restrict__ err,
                                long long* __restrict__ xchg, long long* __restrict__ flag) {
  for (u32 i = threadIdx.x; i < W * (K + 1); i += blockDim.x) {
    const u32 d = i / (K + 1), k = i - d * (K + 1);
    xchg[i] = k < K ? (long long)gh[k * W + d] : failed;
  }
  if (threadIdx.x == 0) flag[0] = (err && err[0]) ? 1 : 0;
}

}  // namespace rc
}  // namespace mr

using namespace mr;

static inline unsigned rc_grid(u64 n, unsigned cap = 8192) {
  u64 g = (n + 255) / 256;
  return (unsigned)(g < 1 ? 1 : (g > cap ? cap : g));
}

// in / out need only be 4-byte aligned (rows of a slice): the kernel takes
// their 16-byte aligned bases and the head bytes before them
template <int C, int R, bool PIPE>
static void launch_gather16_t(const void* in, u64 nin, const void* perm, u64 n, int rb, void* out, hipStream_t s) {
  const u64 nb = (n + R - 1) / R;
  const unsigned g = (unsigned)(nb < 65536 ? nb : 65536);
  const u32 ih = (u32)((uintptr_t)in & 15), oh = (u32)((uintptr_t)out & 15);
  if (ih | oh)
    hipLaunchKernelGGL((rc::rec_gather16_kernel<C, R, PIPE, true>), dim3(g), dim3(256), 0, s, (const u8*)in - ih,
                       nin, (const u32*)perm, n, (u32)rb, (u8*)out - oh, ih, oh);
  else
    hipLaunchKernelGGL((rc::rec_gather16_kernel<C, R, PIPE, false>), dim3(g), dim3(256), 0, s, (const u8*)in, nin,
                       (const u32*)perm, n, (u32)rb, (u8*)out, 0u, 0u);
}

static bool g_gather_pipe = true;  // mr_rec_gather mode 2 forces the unpipelined form (A/B)
// rows per workgroup batch (mr_rec_gather_set_rows): 256 (LDS image of 28 KiB
// for 100-byte rows: 5 workgroups = 20 waves per CU) or 128 (14 KiB: the CU
// fills to 8 waves per SIMD, more row loads in flight)
static int g_gather_rows = 256;

template <int C>
static void launch_gather16(const void* in, u64 nin, const void* perm, u64 n, int rb, void* out, hipStream_t s) {
  constexpr int RD = C <= 8 ? 256 : 128;
  if (g_gather_rows == 128 && RD == 256) {
    if (g_gather_pipe) launch_gather16_t<C, 128, true>(in, nin, perm, n, rb, out, s);
    else launch_gather16_t<C, 128, false>(in, nin, perm, n, rb, out, s);
    return;
  }
  if (g_gather_pipe)
    launch_gather16_t<C, RD, true>(in, nin, perm, n, rb, out, s);
  else
    launch_gather16_t<C, RD, false>(in, nin, perm, n, rb, out, s);
}

extern "C" {

// ghist: null, or a zeroed u32[8][256] that receives the digit histograms of k32
int mr_rec_keys32(const void* rec, u64 n, int rb, int kb, void* k32, void* ghist, hipStream_t s) {
  if (n == 0) return 0;
  if (rb <= 0 || kb <= 0 || kb > rb || kb > 16) return -1;
  hipLaunchKernelGGL(rc::rec_keys32_kernel, dim3(rc_grid(n, ghist ? 2048 : 8192)), dim3(256), 0, s, (const u8*)rec, n,
                     rb, kb, (u32*)k32, (u32*)ghist);
  return (int)hipGetLastError();
}

int mr_rec_keys(const void* rec, u64 n, int rb, int kb, void* hi, void* lo, hipStream_t s) {
  if (n == 0) return 0;
  if (rb <= 0 || kb <= 0 || kb > rb || kb > 16) return -1;
  hipLaunchKernelGGL(rc::rec_keys_kernel, dim3(rc_grid(n)), dim3(256), 0, s, (const u8*)rec, n, rb, kb, (u64*)hi,
                     (u64*)lo);
  return (int)hipGetLastError();
}

// ws: u64 scratch of 1 + ws_cap words (a run counter, then run starts)
// ws: u64 scratch of mr_rec_tie_ws_words(n, ws_cap) words: a run counter,
// ws_cap run starts (runs of 3+), then the scan's per-block counts and
// segments (u32).
u64 mr_rec_tie_ws_words(u64 n, u64 ws_cap) {
  const u64 g = (n + rc::TS_POS - 1) / rc::TS_POS;
  return 1 + ws_cap + (g + g * rc::TS_CAP + 1) / 2 + 1;
}

int mr_rec_tie_fixup(const void* sk, void* perm, const void* rec, u64 n, int rb, int kb, void* bad, void* ws,
                     u64 ws_cap, hipStream_t s) {
  if (n < 2 || kb <= 4) return 0;  // kb <= 4: the prefix is the whole key
  u64* w = (u64*)ws;
  (void)hipMemsetAsync(w, 0, sizeof(u64), s);
  const u64 g = (n + rc::TS_POS - 1) / rc::TS_POS;
  if (g > 0x7FFFFFFFull) return -1;
  u32* counts = reinterpret_cast<u32*>(w + 1 + ws_cap);
  u32* seg = counts + g;
  hipLaunchKernelGGL(rc::rec_tie_scan_kernel, dim3((unsigned)g), dim3(256), 0, s, (const u32*)sk, n, counts, seg,
                     (u32*)bad);
  hipLaunchKernelGGL(rc::rec_tie_fix_kernel, dim3((unsigned)g), dim3(256), 0, s, (const u32*)sk, (u32*)perm,
                     (const u8*)rec, n, rb, kb, (const u32*)counts, (const u32*)seg, (u32*)bad, w + 1,
                     (unsigned long long*)w, ws_cap);
  hipLaunchKernelGGL(rc::rec_tie_runs_kernel, dim3(256), dim3(64), 0, s, (const u32*)sk, (u32*)perm, (const u8*)rec,
                     n, rb, kb, (u32*)bad, (const u64*)(w + 1), (const unsigned long long*)w, ws_cap);
  return (int)hipGetLastError();
}

// nin: rows of `in` (permutation entries >= nin read row 0).  mode: 0 = the
// 16-byte LDS-staged gather where the shape allows it, 1 = the dword gather
// (A/B probes and tests of both paths).
int mr_rec_gather_set_rows(int rows) {
  if (rows != 128 && rows != 256) return -1;
  g_gather_rows = rows;
  return 0;
}

int mr_rec_gather(const void* in, u64 nin, const void* perm, u64 n, int rb, void* out, int mode, hipStream_t s) {
  if (n == 0) return 0;
  if (nin == 0) return -1;
  if (rb & 3) {
    hipLaunchKernelGGL(rc::rec_gather_bytes_kernel, dim3(rc_grid(n * (u64)rb, 16384)), dim3(256), 0, s,
                       (const u8*)in, nin, (const u32*)perm, n, (u64)rb, (u8*)out);
    return (int)hipGetLastError();
  }
  const bool aligned = (((uintptr_t)in | (uintptr_t)out) & 3) == 0;  // (see launch_gather16_t)
  g_gather_pipe = mode != 2;
  if (mode == 2) mode = 0;
  if (mode == 0 && aligned && rb >= 16 && rb <= 244) {
    switch ((rb + 27) / 16) {
      case 2: launch_gather16<2>(in, nin, perm, n, rb, out, s); break;
      case 3: launch_gather16<3>(in, nin, perm, n, rb, out, s); break;
      case 4: launch_gather16<4>(in, nin, perm, n, rb, out, s); break;
      case 5: launch_gather16<5>(in, nin, perm, n, rb, out, s); break;
      case 6: launch_gather16<6>(in, nin, perm, n, rb, out, s); break;
      case 7: launch_gather16<7>(in, nin, perm, n, rb, out, s); break;
      case 8: launch_gather16<8>(in, nin, perm, n, rb, out, s); break;
      case 9: launch_gather16<9>(in, nin, perm, n, rb, out, s); break;
      case 10: launch_gather16<10>(in, nin, perm, n, rb, out, s); break;
      case 11: launch_gather16<11>(in, nin, perm, n, rb, out, s); break;
      case 12: launch_gather16<12>(in, nin, perm, n, rb, out, s); break;
      case 13: launch_gather16<13>(in, nin, perm, n, rb, out, s); break;
      case 14: launch_gather16<14>(in, nin, perm, n, rb, out, s); break;
      case 15: launch_gather16<15>(in, nin, perm, n, rb, out, s); break;
      default: launch_gather16<16>(in, nin, perm, n, rb, out, s); break;
    }
    return (int)hipGetLastError();
  }
  const u32 words = (u32)(rb >> 2);
  const unsigned g = rc_grid(n * words, 16384);
  if (words == 25)
    hipLaunchKernelGGL((rc::rec_gather_kernel<25, 8>), dim3(g), dim3(256), 0, s, (const u32*)in, nin,
                       (const u32*)perm, n, words, (u32*)out);
  else
    hipLaunchKernelGGL((rc::rec_gather_kernel<0, 8>), dim3(g), dim3(256), 0, s, (const u32*)in, nin,
                       (const u32*)perm, n, words, (u32*)out);
  return (int)hipGetLastError();
}

// ghist: zeroed u32 [>= 256]; K * W <= 256 buckets, nsplit = R * K - 1 <= 1023
int mr_rec_bucket32(const void* k32, u64 n, const void* split, u32 nsplit, u32 K, u32 W, void* bucket, void* ghist,
                    hipStream_t s) {
  if (n == 0) return 0;
  if (nsplit > 1024 || K == 0 || W == 0 || (u64)K * W > 256 || (nsplit + 1 + K - 1) / K > W) return -1;
  hipLaunchKernelGGL(rc::rec_bucket32_kernel, dim3(rc_grid(n, 2048)), dim3(256), 0, s, (const u32*)k32, n,
                     (const u32*)split, nsplit, K, W, (u32*)bucket, (u32*)ghist);
  return (int)hipGetLastError();
}

// ghist: zeroed u32 [>= 1024]
int mr_rec_hist32(const void* k32, u64 n, void* ghist, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(rc::rec_hist32_kernel, dim3(rc_grid(n, 2048)), dim3(256), 0, s, (const u32*)k32, n,
                     (u32*)ghist);
  return (int)hipGetLastError();
}

int mr_rec_sample32(const void* k32, u64 n, u32 k, u64 seed, void* out, hipStream_t s) {
  if (k == 0) return 0;
  hipLaunchKernelGGL(rc::rec_sample32_kernel, dim3((k + 255) / 256), dim3(256), 0, s, (const u32*)k32, n, k, seed,
                     (long long*)out);
  return (int)hipGetLastError();
}

// srt: N sorted int64 (negatives = no sample); sp: R - 1 u32
int mr_rec_pick(const void* srt, u64 N, u32 R, void* sp, hipStream_t s) {
  if (R <= 1) return 0;
  if (N == 0) return -1;
  hipLaunchKernelGGL(rc::rec_pick_kernel, dim3(1), dim3(256), 0, s, (const long long*)srt, N, R, (u32*)sp);
  return (int)hipGetLastError();
}

int mr_rec_xchg(const void* gh, u32 K, u32 W, long long failed, const void* err, void* xchg, void* flag,
                hipStream_t s) {
  if ((u64)K * W > 256) return -1;
  hipLaunchKernelGGL(rc::rec_xchg_kernel, dim3(1), dim3(256), 0, s, (const u32*)gh, K, W, failed, (const u32*)err,
                     (long long*)xchg, (long long*)flag);
  return (int)hipGetLastError();
}

int mr_rec_dest32(const void* k32, u64 n, const void* split, u32 nsplit, void* dest, hipStream_t s) {
  if (n == 0) return 0;
  if (nsplit > 1024) return -1;
  hipLaunchKernelGGL(rc::rec_dest32_kernel, dim3(rc_grid(n)), dim3(256), 0, s, (const u32*)k32, n, (const u32*)split,
                     nsplit, (u32*)dest);
  return (int)hipGetLastError();
}

}  // extern "C"
