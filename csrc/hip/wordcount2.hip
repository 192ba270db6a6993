// wordcount2.hip — second-generation fused word-count map kernel (gfx950).
//
// Same contract as wc_map_kernel (wordcount.hip): tokenize a byte stream on
// Lua-%s whitespace, build exact 128-bit keys, combine in LDS, fold partials
// into the HBM table (reference hot loops K1-K5: examples/WordCount/mapfn.lua,
// job.lua:83-97, job.lua:92-96).  What changes, and why (rocprof of v1: 90 % of
// the step in the map kernel at ~38 GB/s):
//   * no per-byte dependent LDS loops: every thread turns its 16 staged bytes
//     into a 16-bit whitespace mask stored as an LDS bitmap; a token's end is a
//     count-trailing-zeros on one or two bitmap words, and its key is packed
//     from five aligned ds_read_b32 + funnel shifts + bswap (no byte loop);
//   * 512-thread workgroups (8 wave64) on 8 KiB tiles, 4096-slot LDS table
//     (112 KiB, 1 workgroup / CU) so a 64 KiB chunk's vocabulary fits;
//   * tokens that miss the LDS table (cold words once it is 3/4 full) are not
//     inserted into HBM with a dependent probe chain inside the divergent token
//     loop; they are appended to an overflow buffer (one coalesced atomic per
//     wave) and folded by a separate full-occupancy kernel.
#include <hip/hip_runtime.h>
#include "mr_common.h"
#include "hashtab.h"

namespace mr {
namespace v2 {

constexpr int T = 512;
constexpr int SEG = 16;
constexpr int TILE = T * SEG;              // 8192 bytes
constexpr int PAD = 16;                    // txt[PAD-1] = byte before the tile
constexpr int HALO = 64;                   // staged bytes of the next tile
constexpr int STAGED = TILE + HALO;        // bitmap covers [0, STAGED)
constexpr int TXT = PAD + STAGED + 32;     // + slack for word reads
constexpr int WSW = STAGED / 32 + 2;       // bitmap words (+2 all-ones pad)
constexpr int SLOTS = 4096;
constexpr int CLAIM_LIMIT = SLOTS * 3 / 4;
constexpr int PROBES = 32;

enum Mode : int { FULL = 0, TOKENIZE_ONLY = 1, NO_GLOBAL = 2, NO_OVERFLOW = 3, STAGED_FLUSH = 4 };

struct Lds {
  u8 txt[TXT];
  u32 ws[WSW];
  u32 tag[SLOTS];
  u32 cnt[SLOTS];
  u32 rep[SLOTS];  // local offset (16 bits) | len (16 bits) << 16
  u64 lo[SLOTS];
  u64 hi[SLOTS];
  u32 nclaimed;
};

struct Ovf {
  u64* hi;
  u64* lo;
  u64* rep;
  u64 cap;
  unsigned long long* counter;
  u32* cnt;  // per-entry count (STAGED mode); null: every entry counts 1
};

__device__ __forceinline__ u32 ws_mask_word(u32 w) {
  u32 m = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) m |= (is_ws((w >> (8 * j)) & 0xFFu) ? 1u : 0u) << j;
  return m;
}

__device__ __forceinline__ u32 funnel(u32 a, u32 b, u32 r8) {
  // bytes starting at byte r of the 8-byte little-endian pair (a, b)
  return r8 ? ((a >> r8) | (b << (32 - r8))) : a;
}

__device__ u64 long_lo_global(const u8* text, u64 p0, u64 len) {
  u64 h = long_hash_init(len);
  for (u64 w = 0; w < len; w += 8) {
    u64 word = 0;
    const u64 n = (len - w) < 8 ? (len - w) : 8;
    for (u64 j = 0; j < n; ++j) word |= (u64)text[p0 + w + j] << (8 * j);
    h = long_hash_step(h, word);
  }
  return long_lo(h);
}

__device__ __forceinline__ bool lds_insert(Lds& L, u64 hi, u64 lo, u32 rep) {
  // cheap 64-bit mix: packed keys keep their bytes in the HIGH bits (short
  // words have all-zero low words), so fold high into low before using bits
  u64 h = hi ^ (lo * 0x9E3779B97F4A7C15ull);
  h ^= h >> 31;
  h *= 0xC2B2AE3D27D4EB4Full;
  h ^= h >> 29;
  const u32 tag = (u32)(h >> 32) | 1u;
  u32 slot = (u32)h & (SLOTS - 1);
  int probes = 0;
  while (probes < PROBES) {
    u32 cur = __hip_atomic_load(&L.tag[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (cur == 0) {
      if (__hip_atomic_load(&L.nclaimed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= (u32)CLAIM_LIMIT)
        return false;
      u32 expected = 0;
      if (__hip_atomic_compare_exchange_strong(&L.tag[slot], &expected, tag, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP)) {
        L.hi[slot] = hi;
        L.rep[slot] = rep;
        __hip_atomic_fetch_add(&L.cnt[slot], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(&L.nclaimed, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_store(&L.lo[slot], lo, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        return true;
      }
      cur = expected;
    }
    if (cur == tag) {
      const u64 l = __hip_atomic_load(&L.lo[slot], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (l == 0) continue;  // claimer has not published yet
      if (l == lo && L.hi[slot] == hi) {
        __hip_atomic_fetch_add(&L.cnt[slot], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return true;
      }
    }
    slot = (slot + 1) & (SLOTS - 1);
    ++probes;
  }
  return false;
}

__device__ __forceinline__ u32 overflow_push(const Ovf& o, const GTab& g, u64 hi, u64 lo, u64 rep) {
  const unsigned long long idx = atomicAdd(o.counter, 1ull);
  if (idx < o.cap) {
    o.hi[idx] = hi;
    o.lo[idx] = lo;
    o.rep[idx] = rep;
    if (o.cnt) o.cnt[idx] = 1u;
    return 0;
  }
  return gtab_insert(g, hi, lo, 1, rep, OP_SUM) == 2;
}

template <int MODE>
__global__ void __launch_bounds__(T) wc_map2_kernel(const u8* __restrict__ text, u64 nbytes, u64 chunk_bytes,
                                                    u64 rep_base, GTab g, Ovf ovf, int aligned, u64* sink) {
  __shared__ __attribute__((aligned(16))) Lds L;
  const int t = threadIdx.x;
  const u64 chunk_begin = (u64)blockIdx.x * chunk_bytes;
  if (chunk_begin >= nbytes) return;
  const u64 chunk_end = min(chunk_begin + chunk_bytes, nbytes);
  if (MODE != TOKENIZE_ONLY) {
    for (int s = t; s < SLOTS; s += T) {
      L.tag[s] = 0;
      L.cnt[s] = 0;
      L.lo[s] = 0;
    }
  }
  if (t == 0) {
    L.nclaimed = 0;
    L.txt[PAD - 1] = chunk_begin > 0 ? text[chunk_begin - 1] : (u8)' ';
    L.ws[WSW - 2] = 0xFFFFFFFFu;
    L.ws[WSW - 1] = 0xFFFFFFFFu;
  }
  u64 acc = 0;
  u32 claims = 0;
  u16* ws16 = reinterpret_cast<u16*>(L.ws);
  const u32* txt32 = reinterpret_cast<const u32*>(L.txt);
  for (u64 tile_base = chunk_begin; tile_base < chunk_end; tile_base += TILE) {
    // ---- stage 16 bytes per thread + the halo, and the whitespace bitmap
    {
      const u64 gpos = tile_base + (u64)t * SEG;
      uint4 q;
      if (aligned && gpos + SEG <= nbytes) {
        q = *reinterpret_cast<const uint4*>(text + gpos);
      } else {
        u32 w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          w[k] = 0;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const u64 p = gpos + 4 * k + j;
            w[k] |= (p < nbytes ? (u32)text[p] : 32u) << (8 * j);
          }
        }
        q = make_uint4(w[0], w[1], w[2], w[3]);
      }
      *reinterpret_cast<uint4*>(L.txt + PAD + t * SEG) = q;
      ws16[t] = (u16)(ws_mask_word(q.x) | (ws_mask_word(q.y) << 4) | (ws_mask_word(q.z) << 8) |
                      (ws_mask_word(q.w) << 12));
      if (t < HALO / SEG) {
        const u64 gh = tile_base + TILE + (u64)t * SEG;
        u32 w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          w[k] = 0;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const u64 p = gh + 4 * k + j;
            w[k] |= (p < nbytes ? (u32)text[p] : 32u) << (8 * j);
          }
        }
        *reinterpret_cast<uint4*>(L.txt + PAD + TILE + t * SEG) = make_uint4(w[0], w[1], w[2], w[3]);
        ws16[T + t] = (u16)(ws_mask_word(w[0]) | (ws_mask_word(w[1]) << 4) | (ws_mask_word(w[2]) << 8) |
                            (ws_mask_word(w[3]) << 12));
      }
    }
    __syncthreads();
    // ---- tokens starting in this thread's segment
    const u64 seg_base = tile_base + (u64)t * SEG;
    if (seg_base < chunk_end) {
      const u32 m = ws16[t];
      const u32 prev_ws = t ? ((ws16[t - 1] >> 15) & 1u) : (is_ws(L.txt[PAD - 1]) ? 1u : 0u);
      u32 starts = (~m) & ((m << 1) | prev_ws) & 0xFFFFu;
      const u64 lim_own = chunk_end - seg_base;
      if (lim_own < 16) starts &= (1u << lim_own) - 1u;
      while (starts) {
        const int i = __builtin_ctz(starts);
        starts &= starts - 1;
        const u32 p = (u32)t * SEG + i;  // tile-relative start
        // end = first whitespace bit after p
        u32 q = p + 1;
        u32 wd = L.ws[q >> 5] >> (q & 31);
        u32 end;
        if (wd) {
          end = q + __builtin_ctz(wd);
        } else {
          u32 k = (q >> 5) + 1;
          while (L.ws[k] == 0) ++k;  // pad words are all ones
          end = 32 * k + __builtin_ctz(L.ws[k]);
        }
        u64 len = end - p;
        const u64 gpos = tile_base + p;
        // pack the first 16 bytes from five aligned words
        const u32 b = PAD + p;
        const u32 a = b >> 2;
        const u32 r8 = (b & 3u) * 8u;
        const u32 x0 = txt32[a], x1 = txt32[a + 1], x2 = txt32[a + 2], x3 = txt32[a + 3], x4 = txt32[a + 4];
        const u64 le_hi = (u64)funnel(x0, x1, r8) | ((u64)funnel(x1, x2, r8) << 32);
        const u64 le_lo = (u64)funnel(x2, x3, r8) | ((u64)funnel(x3, x4, r8) << 32);
        u64 hi = __builtin_bswap64(le_hi);
        u64 lo;
        if (end >= (u32)STAGED) {  // runs past the staged halo: measure from global memory
          u64 pe = tile_base + STAGED;
          while (pe < nbytes && !is_ws(text[pe])) ++pe;
          len = pe - gpos;
        }
        if (len <= (u64)PACK_MAX) {
          if (len < 8) hi &= ~0ull << (8 * (8 - len));
          lo = len > 8 ? (__builtin_bswap64(le_lo) & (~0ull << (8 * (16 - len)))) : 0ull;
          lo |= len;
        } else {
          lo = long_lo_global(text, gpos, len);
        }
        if (MODE == TOKENIZE_ONLY) {
          acc ^= hi * 31 + lo;
          continue;
        }
        const u64 grep = make_rep(rep_base + gpos, len);
        const bool ok = len < 65536 && lds_insert(L, hi, lo, (u32)(gpos - chunk_begin) | ((u32)len << 16));
        if (!ok && (MODE == FULL || MODE == STAGED_FLUSH)) claims += overflow_push(ovf, g, hi, lo, grep);
      }
    }
    __syncthreads();
    if (t == 0) L.txt[PAD - 1] = L.txt[PAD + TILE - 1];
    __syncthreads();
  }
  if (MODE == TOKENIZE_ONLY) {
    if (acc == 0x12345) sink[0] = acc;  // keep the tokenizer live
    return;
  }
  if (MODE == NO_GLOBAL) {
    if (t == 0 && L.nclaimed == 0x7FFFFFFF) sink[0] = 1;
    return;
  }
  if (MODE == STAGED_FLUSH) {
    // append the block's distinct keys (with counts) to the staging buffer —
    // coalesced stores, ONE global atomic per block — and leave the HBM-table
    // inserts to a full-occupancy kernel (this kernel runs 1 workgroup/CU, too
    // few waves to hide the latency of dependent global atomics)
    constexpr int PER = SLOTS / T;
    u32 mine = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) mine += L.tag[t * PER + k] != 0;
    const int lane = t & 63, wave = t >> 6;
    u32 incl = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const u32 v = __shfl_up(incl, o);
      if (lane >= o) incl += v;
    }
    __shared__ u32 wsum[T / 64];
    __shared__ unsigned long long base;
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    u32 before = 0, total = 0;
#pragma unroll
    for (int w = 0; w < T / 64; ++w) {
      before += w < wave ? wsum[w] : 0u;
      total += wsum[w];
    }
    if (t == 0) base = atomicAdd(ovf.counter, (unsigned long long)total);
    __syncthreads();
    unsigned long long pos = base + before + incl - mine;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int s = t * PER + k;
      if (L.tag[s] == 0) continue;
      const u32 r = L.rep[s];
      const u64 rp = make_rep(rep_base + chunk_begin + (r & 0xFFFFu), r >> 16);
      if (pos < ovf.cap) {
        ovf.hi[pos] = L.hi[s];
        ovf.lo[pos] = L.lo[s];
        ovf.rep[pos] = rp;
        ovf.cnt[pos] = L.cnt[s];
      } else {
        claims += gtab_insert(g, L.hi[s], L.lo[s], (long long)L.cnt[s], rp, OP_SUM) == 2;
      }
      ++pos;
    }
    gtab_count_claims(g, claims);
    return;
  }
  for (int s = t; s < SLOTS; s += T) {
    if (L.tag[s] != 0) {
      const u32 r = L.rep[s];
      claims += gtab_insert(g, L.hi[s], L.lo[s], (long long)L.cnt[s],
                            make_rep(rep_base + chunk_begin + (r & 0xFFFFu), r >> 16), OP_SUM) == 2;
    }
  }
  gtab_count_claims(g, claims);
}

__global__ void __launch_bounds__(256) ovf_agg_kernel(Ovf o, GTab g) {
  const unsigned long long n0 = *o.counter;
  const u64 n = n0 < o.cap ? n0 : o.cap;
  const u64 stride = (u64)gridDim.x * blockDim.x;
  u32 claims = 0;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    claims += gtab_insert(g, o.hi[i], o.lo[i], o.cnt ? (long long)o.cnt[i] : 1ll, o.rep[i], OP_SUM) == 2;
  gtab_count_claims(g, claims);
}

}  // namespace v2
}  // namespace mr

using namespace mr;

extern "C" {

// mode: 0 full, 1 tokenize only, 2 LDS only, 3 LDS + flush (no overflow) —
// modes 1-3 exist for ablation timing only (their tables are incomplete).
int mr_wc_map2(const void* text, u64 nbytes, u64 chunk_bytes, u64 rep_base, void* tag, void* hi, void* lo, void* val,
               void* rep, void* ctrl, u64 cap, void* ovf_hi, void* ovf_lo, void* ovf_rep, u64 ovf_cap,
               void* ovf_counter, int mode, void* ovf_cnt, hipStream_t stream) {
  if (nbytes == 0) return 0;
  if (chunk_bytes % v2::TILE || chunk_bytes > 65536) return -1;
  GTab g;
  g.tag = (u64*)tag;
  g.hi = (u64*)hi;
  g.lo = (u64*)lo;
  g.val = (long long*)val;
  g.rep = (u64*)rep;
  g.ctrl = (u32*)ctrl;
  g.mask = cap - 1;
  v2::Ovf o{(u64*)ovf_hi, (u64*)ovf_lo, (u64*)ovf_rep, ovf_cap, (unsigned long long*)ovf_counter, (u32*)ovf_cnt};
  if (mode == 4 && !ovf_cnt) return -1;
  const u64 nblocks = (nbytes + chunk_bytes - 1) / chunk_bytes;
  const int aligned = ((uintptr_t)text & 15) == 0;
  const u8* tx = (const u8*)text;
  dim3 grid((unsigned)nblocks), block(v2::T);
  switch (mode) {
    case 1: hipLaunchKernelGGL(v2::wc_map2_kernel<1>, grid, block, 0, stream, tx, nbytes, chunk_bytes, rep_base, g, o,
                               aligned, (u64*)ovf_counter); break;
    case 2: hipLaunchKernelGGL(v2::wc_map2_kernel<2>, grid, block, 0, stream, tx, nbytes, chunk_bytes, rep_base, g, o,
                               aligned, (u64*)ovf_counter); break;
    case 3: hipLaunchKernelGGL(v2::wc_map2_kernel<3>, grid, block, 0, stream, tx, nbytes, chunk_bytes, rep_base, g, o,
                               aligned, (u64*)ovf_counter); break;
    case 4:
      hipLaunchKernelGGL(v2::wc_map2_kernel<4>, grid, block, 0, stream, tx, nbytes, chunk_bytes, rep_base, g, o,
                         aligned, (u64*)ovf_counter);
      hipLaunchKernelGGL(v2::ovf_agg_kernel, dim3(4096), dim3(256), 0, stream, o, g);
      break;
    default:
      o.cnt = nullptr;
      hipLaunchKernelGGL(v2::wc_map2_kernel<0>, grid, block, 0, stream, tx, nbytes, chunk_bytes, rep_base, g, o,
                         aligned, (u64*)ovf_counter);
      hipLaunchKernelGGL(v2::ovf_agg_kernel, dim3(2048), dim3(256), 0, stream, o, g);
  }
  return (int)hipGetLastError();
}

}  // extern "C"
