// sort.hip — LDS-tiled LSD radix sort, device-wide scans and segmented
// primitives for gfx950 (wave64).
//
// Replaces the reference's ordering/merging hot loops:
//   K6 map-side key sort   utils.lua:123-128 keys_sorted + job.lua:194
//   K9 k-way merge         utils.lua:206-271 merge_iterator + heap.lua:29-70
//   K8 reducer fold        job.lua:264-284 (per merged key)
// Instead of a heap merge of 197 sorted runs per partition, the receiver
// re-sorts the whole received buffer (radix sort is O(n) and bandwidth bound)
// and folds equal keys with a segmented reduce.
//
// Radix pass = 3 launches: per-tile 256-bin histogram (LDS atomics), one
// device-wide exclusive scan over the digit-major [256][tiles] histogram, and a
// stable scatter in which each wave64 ranks its keys with 8 ballots (one per
// digit bit): peers = AND_b (bit_b ? ballot_b : ~ballot_b), rank = popc(peers &
// lanes_below).  Tiles are ITEMS = 16 x 256 keys; keys are visited round by
// round (item = round*256 + thread) so a tile keeps input order (stability).
#include <hip/hip_runtime.h>
#include <cstring>
#include "mr_common.h"

namespace mr {

constexpr int RS_THREADS = 256;
constexpr int RS_ROUNDS = 16;
constexpr int RS_TILE = RS_THREADS * RS_ROUNDS;  // 4096 keys per tile
constexpr int RS_BINS = 256;
constexpr int RS_WAVES = RS_THREADS / 64;

// ---------------------------------------------------------------------------
// Onesweep-style LSD pass: ONE launch per 8-bit digit.
//   * rs_ghist8_kernel computes the global 256-bin histograms of all 8 digits of
//     a u64 word at once (digit counts do not depend on the current order);
//   * rs_onesweep_kernel: tiles are taken in dispatch order from an atomic
//     counter (so every predecessor tile is already resident: no deadlock),
//     each tile publishes its per-digit count as a tagged 64-bit granule
//     {epoch:24 | flag:2 | count:38} (guide §6 G16 R2: the data is the flag),
//     looks back over predecessors for its exclusive prefix, republishes the
//     inclusive prefix, then scatters with the same stable wave64-ballot ranking
//     as the LDS tile ranking.  A digit shared by every key makes the pass a copy.
//   * every spin is bounded (s_sleep + give-up sets err[0]).
constexpr u64 GR_AGG = 1ull, GR_INC = 2ull;

__device__ __forceinline__ u64 gr_pack(u32 epoch, u64 flag, u64 count) {
  return ((u64)(epoch & 0xFFFFFFu) << 40) | (flag << 38) | (count & ((1ull << 38) - 1));
}

template <bool RUNS>
__global__ void __launch_bounds__(RS_THREADS) rs_ghist8_kernel(const u64* keys, u64 n, u32* ghist /*[8][256]*/,
                                                               int d0, int ndigits) {
  // only the digits the sort will visit: a 16-bit word used to pay 6 extra
  // all-in-bin-0 (maximally contended) LDS atomics per key
  __shared__ u32 h[8][RS_BINS];
  const int t = threadIdx.x;
#pragma unroll
  for (int b = 0; b < 8; ++b) h[b][t] = 0;
  __syncthreads();
  // RUNS (caller's hint: keys with runs of equal digits, e.g. posting keys in
  // text order share their line digits over a whole line): a run is counted by
  // its first lane only — same-address LDS atomics from a wave serialise, and
  // ~25-key runs had made this kernel 0.4 ms on 46 M posting keys (0.08 ms
  // run-aggregated).  On random keys the aggregation costs more than it saves
  // (0.27 -> 0.61 ms on 100 M TeraSort keys), hence the hint.  A wave walks its
  // 64 keys as one (uniform loop); the valid lanes are a prefix.
  const u64 stride = (u64)gridDim.x * blockDim.x;
  if constexpr (!RUNS) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + t; i < n; i += stride) {
      const u64 k = keys[i];
#pragma unroll
      for (int b = 0; b < 8; ++b)
        if (b >= d0 && b < ndigits) atomicAdd(&h[b][(k >> (8 * b)) & 0xFF], 1u);
    }
  }
  const int lane = t & 63;
  for (u64 base = (u64)blockIdx.x * blockDim.x + (u64)(t & ~63); RUNS && base < n; base += stride) {
    const u64 i = base + lane;
    const bool valid = i < n;
    const u64 k = valid ? keys[i] : 0ull;
    const u32 nvalid = n - base < 64 ? (u32)(n - base) : 64u;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      if (b >= d0 && b < ndigits) {
        const u32 d = (u32)(k >> (8 * b)) & 0xFFu;
        const u32 prev = __shfl_up(d, 1);
        const bool head = valid && (lane == 0 || d != prev);
        const u64 hm = __ballot(head);
        if (head) {
          const u64 after = lane == 63 ? 0ull : (hm >> (lane + 1));
          const u32 end = after ? (u32)(lane + __ffsll((long long)after)) : nvalid;
          atomicAdd(&h[b][d], end - (u32)lane);
        }
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int b = 0; b < 8; ++b)
    if (b >= d0 && b < ndigits && h[b][t]) atomicAdd(&ghist[b * RS_BINS + t], h[b][t]);
}

// Inclusive scan of one value per thread over a 256-thread block: wave64
// shuffles, then the 4 wave totals through LDS (2 barriers instead of the 16
// of a Hillis-Steele loop over LDS).  `tmp` is 4 words of LDS.
__device__ __forceinline__ u32 block_scan_256(u32 v, u32* tmp) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const u32 y = __shfl_up(v, o);
    if (lane >= o) v += y;
  }
  __syncthreads();  // tmp may still be read by a previous scan
  if (lane == 63) tmp[wave] = v;
  __syncthreads();
  u32 add = 0;
#pragma unroll
  for (int w = 0; w < RS_WAVES; ++w) add += w < wave ? tmp[w] : 0u;
  return v + add;
}

// ROUNDS: tiles of 256 x ROUNDS keys (onesweep_rounds below): 4 (1024-key
// tiles) below ONESWEEP_SMALL keys, where a pass is one tile's latency and
// 4096-key tiles left most CUs idle (54k keys = 14 tiles); 16 or more above.
constexpr u64 ONESWEEP_SMALL = 1ull << 18;
// K: u64 keys, or u32 keys (TeraSort's 32-bit key prefixes: a third less
// traffic per pass than u64 keys with u32 values).
template <typename K, typename V, int ROUNDS>
__global__ void __launch_bounds__(RS_THREADS) rs_onesweep_kernel(const K* keys_in, const V* vals_in, K* keys_out,
                                                                 V* vals_out, u64 n, int shift, const u32* ghist,
                                                                 u64* granules, u32* tile_counter, u32 epoch,
                                                                 u32* err, int iota, int debug_fail) {
  constexpr int RS_TILE = RS_THREADS * ROUNDS;
  constexpr int RS_ROUNDS = ROUNDS;
  // iota: vals_in is absent and the value of key i is i (first pass of a
  // permutation sort; saves the separate iota launch).
  // Each wave ranks its own contiguous quarter of the tile (16 rounds of 64
  // keys) against WAVE-PRIVATE digit counters in LDS — no block barrier inside
  // the rounds (the first version paid 3 barriers per round).  The tile
  // histogram falls out of the four wave counters; keys (and values) are then
  // placed in an LDS image of the tile in digit order and streamed out so
  // consecutive lanes write consecutive addresses of one digit run.
  constexpr int SUB = RS_TILE / RS_WAVES;  // keys per wave
  __shared__ K sk[RS_TILE];
  __shared__ V sv[RS_TILE];
  __shared__ u32 wc[RS_WAVES][RS_BINS];
  __shared__ u32 gout[RS_BINS];
  __shared__ u32 sh_tile;
  __shared__ u32 sh_uniform;
  __shared__ u32 wsum[RS_WAVES];
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  if (t == 0) {
    sh_tile = atomicAdd(tile_counter, 1u);
    sh_uniform = 0;
  }
#pragma unroll
  for (int w = 0; w < RS_WAVES; ++w) wc[w][t] = 0;
  // exclusive scan of the global histogram (digit base offsets)
  const u32 gcount = ghist[t];
  __syncthreads();
  if (gcount == n) sh_uniform = 1;
  const u32 gbase = block_scan_256(gcount, wsum) - gcount;
  __syncthreads();
  const u32 tile = sh_tile;
  const u64 t0 = (u64)tile * RS_TILE;
  if (sh_uniform) {  // every key has this digit: order unchanged
    for (int r = 0; r < RS_ROUNDS; ++r) {
      const u64 i = t0 + (u64)r * RS_THREADS + t;
      if (i < n) {
        keys_out[i] = keys_in[i];
        if (vals_in) vals_out[i] = vals_in[i];
        else if (iota) vals_out[i] = (V)i;
      }
    }
    return;
  }
  const bool has_v = vals_in != nullptr || iota;
  // this wave's keys: tile[wave*SUB + r*64 + lane]
  const u64 w0 = t0 + (u64)wave * SUB;
  K kr[RS_ROUNDS];
  V vr[RS_ROUNDS];
#pragma unroll
  for (int r = 0; r < RS_ROUNDS; ++r) {
    const u64 i = w0 + (u64)r * 64 + lane;
    kr[r] = i < n ? keys_in[i] : 0;
    vr[r] = (i < n && vals_in) ? vals_in[i] : (iota ? (V)i : V{});
  }
  const unsigned long long below = (1ull << lane) - 1ull;
  u32 myrank[RS_ROUNDS];
  u32* mywc = wc[wave];
#pragma unroll
  for (int r = 0; r < RS_ROUNDS; ++r) {
    const u64 i = w0 + (u64)r * 64 + lane;
    const bool valid = i < n;
    const u32 d = (u32)((kr[r] >> shift) & 0xFF);
    unsigned long long peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const unsigned long long m = __ballot((d >> b) & 1u);
      peers &= ((d >> b) & 1u) ? m : ~m;
    }
    const u32 before = valid ? mywc[d] : 0u;
    myrank[r] = before + (u32)__popcll(peers & below);
    // every lane has read its counter before the leader updates it (LDS ops of
    // one wave complete in order)
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    if (valid && (peers & below) == 0) mywc[d] = before + (u32)__popcll(peers);
  }
  __syncthreads();
  // tile histogram + per-wave offsets for digit t
  u32 cnt_w[RS_WAVES];
  u32 mine = 0;
#pragma unroll
  for (int w = 0; w < RS_WAVES; ++w) {
    cnt_w[w] = wc[w][t];
    mine += cnt_w[w];
  }
  u64* G = granules + (u64)tile * RS_BINS;
  __hip_atomic_store(&G[t], gr_pack(epoch, tile == 0 ? GR_INC : GR_AGG, mine), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
  const u32 lbase = block_scan_256(mine, wsum) - mine;
  {
    u32 off = lbase;
#pragma unroll
    for (int w = 0; w < RS_WAVES; ++w) {
      wc[w][t] = off;  // now: LDS start of wave w's keys of digit t
      off += cnt_w[w];
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < RS_ROUNDS; ++r) {
    const u64 i = w0 + (u64)r * 64 + lane;
    if (i < n) {
      const u32 d = (u32)((kr[r] >> shift) & 0xFF);
      const u32 pos = mywc[d] + myrank[r];
      sk[pos] = kr[r];
      if (has_v) sv[pos] = vr[r];
    }
  }
  // decoupled look-back for this tile's global prefix of digit t
  u64 excl = 0;
  if (tile > 0) {
    long long j = (long long)tile - 1;
    u32 spins = 0;
    if (debug_fail && tile == 1) {  // test knob (mr_sort_debug_fail): this tile gives up at once
      atomicOr(err, 1u);
      j = -1;
    }
    while (j >= 0) {
      const u64 g = __hip_atomic_load(&granules[(u64)j * RS_BINS + t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const u32 ep = (u32)(g >> 40);
      const u64 fl = (g >> 38) & 3ull;
      if (ep != (epoch & 0xFFFFFFu) || fl == 0) {
        if (++spins > (1u << 22)) {
          atomicOr(err, 1u);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      excl += g & ((1ull << 38) - 1);
      if (fl == GR_INC) break;
      --j;
    }
    __hip_atomic_store(&G[t], gr_pack(epoch, GR_INC, excl + mine), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  gout[t] = gbase + (u32)excl - lbase;  // global pos of LDS index i with digit d = gout[d] + i
  __syncthreads();
  const u32 cnt = (u32)min((u64)RS_TILE, n - t0);
  for (u32 i = t; i < cnt; i += RS_THREADS) {
    const K k = sk[i];
    const u32 pos = gout[(k >> shift) & 0xFF] + i;
    // After a give-up (here or in an earlier pass of the same sort) the input
    // holds rows left over from other data, whose digits no longer match the
    // precomputed histograms: positions can then run past n.  The order is
    // reported invalid through `err`; the writes must still stay in bounds.
    if (pos >= n) continue;
    keys_out[pos] = k;
    if (has_v) vals_out[pos] = sv[i];
  }
}

// ---------------------------------------------------------------------------
// Device-wide exclusive scan (reduce-then-scan, 3 launches).
constexpr int SC_THREADS = 256;
constexpr int SC_ITEMS = 16;
constexpr int SC_TILE = SC_THREADS * SC_ITEMS;

template <typename T>
__device__ __forceinline__ T block_exclusive_scan(T x, T* sh, T* total) {
  // Hillis-Steele over 256 threads in LDS (small; used once per tile).
  const int t = threadIdx.x;
  sh[t] = x;
  __syncthreads();
  for (int o = 1; o < SC_THREADS; o <<= 1) {
    T y = t >= o ? sh[t - o] : (T)0;
    __syncthreads();
    sh[t] += y;
    __syncthreads();
  }
  const T incl = sh[t];
  if (total) *total = sh[SC_THREADS - 1];
  __syncthreads();
  return incl - x;
}

template <typename T>
__global__ void __launch_bounds__(SC_THREADS) scan_reduce_kernel(const T* in, u64 n, T* partials) {
  __shared__ T sh[SC_THREADS];
  const u64 base = (u64)blockIdx.x * SC_TILE;
  T s = 0;
  for (int r = 0; r < SC_ITEMS; ++r) {
    const u64 i = base + (u64)r * SC_THREADS + threadIdx.x;
    if (i < n) s += in[i];
  }
  T tot;
  block_exclusive_scan<T>(s, sh, &tot);
  if (threadIdx.x == 0) partials[blockIdx.x] = tot;
}

template <typename T>
__global__ void __launch_bounds__(SC_THREADS) scan_partials_kernel(T* partials, u64 np, T* total_out) {
  // single block: each thread scans a contiguous strip, then block scan of strips
  __shared__ T sh[SC_THREADS];
  const u64 per = (np + SC_THREADS - 1) / SC_THREADS;
  const u64 b = (u64)threadIdx.x * per;
  T s = 0;
  for (u64 i = b; i < b + per && i < np; ++i) s += partials[i];
  T tot;
  T off = block_exclusive_scan<T>(s, sh, &tot);
  for (u64 i = b; i < b + per && i < np; ++i) {
    T x = partials[i];
    partials[i] = off;
    off += x;
  }
  if (threadIdx.x == 0 && total_out) *total_out = tot;
}

template <typename T>
__global__ void __launch_bounds__(SC_THREADS) scan_apply_kernel(const T* in, u64 n, T* out, const T* partials) {
  __shared__ T sh[SC_THREADS];
  const u64 base = (u64)blockIdx.x * SC_TILE;
  // each thread owns SC_ITEMS contiguous items -> local sums, block scan, rescan
  const u64 my = base + (u64)threadIdx.x * SC_ITEMS;
  T vals[SC_ITEMS];
  T s = 0;
#pragma unroll
  for (int r = 0; r < SC_ITEMS; ++r) {
    const u64 i = my + r;
    vals[r] = i < n ? in[i] : (T)0;
    s += vals[r];
  }
  T off = block_exclusive_scan<T>(s, sh, nullptr) + partials[blockIdx.x];
#pragma unroll
  for (int r = 0; r < SC_ITEMS; ++r) {
    const u64 i = my + r;
    if (i < n) out[i] = off;
    off += vals[r];
  }
}

// ---------------------------------------------------------------------------
__global__ void gather_u64_kernel(const u64* src, const u32* idx, u64* dst, u64 n) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = src[clamp_row(idx[i], n)];
}

__global__ void iota_u32_kernel(u32* dst, u64 n) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = (u32)i;
}

// heads[i] = 1 if (hi,lo)[i] starts a new run (keys sorted)
__global__ void segment_heads_kernel(const u64* hi, const u64* lo, u64 n, u32* heads) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    heads[i] = (i == 0 || hi[i] != hi[i - 1] || (lo && lo[i] != lo[i - 1])) ? 1u : 0u;
  }
}

// segment id (inclusive scan of heads - 1) is computed by the caller as
// exclusive_scan(heads) + heads - 1; here fold values per segment with atomics
// (segments are contiguous, so contention is bounded by a segment's length).
__global__ void segment_fold_kernel(const u32* seg_excl, const u32* heads, const long long* vals, u64 n, int op,
                                    long long* out) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const u32 s = seg_excl[i] + heads[i] - 1u;
    const long long v = vals ? vals[i] : 1ll;
    if (op == OP_MIN) atomicMin(&out[s], v);
    else if (op == OP_MAX) atomicMax(&out[s], v);
    else atomicAdd((unsigned long long*)&out[s], (unsigned long long)v);
  }
}

// unique keys: out[s] = key[i] for every head i
__global__ void segment_keys_kernel(const u32* seg_excl, const u32* heads, const u64* hi, const u64* lo,
                                    const u64* rep, u64 n, u64* out_hi, u64* out_lo, u64* out_rep, u64* out_start) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    if (heads[i]) {
      const u32 s = seg_excl[i];
      out_hi[s] = hi[i];
      if (lo) out_lo[s] = lo[i];
      if (rep) out_rep[s] = rep[i];
      if (out_start) out_start[s] = i;
    }
  }
}

// histogram of small-integer ids (partition / destination counts)
__global__ void bincount_kernel(const u32* ids, u64 n, u32 nbins, long long* counts) {
  extern __shared__ u32 sh[];
  for (u32 b = threadIdx.x; b < nbins; b += blockDim.x) sh[b] = 0;
  __syncthreads();
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) atomicAdd(&sh[ids[i]], 1u);
  __syncthreads();
  for (u32 b = threadIdx.x; b < nbins; b += blockDim.x)
    if (sh[b]) atomicAdd((unsigned long long*)&counts[b], (unsigned long long)sh[b]);
}

// After sorting by a composite key c = (part << 56) | (hi >> 8), finish the
// (part, hi, lo) order: runs of equal c (same partition and same first 7 key
// bytes) are insertion-sorted by (hi & 0xFF, lo) together with their payload
// columns.  Runs longer than FIX_MAX set *bad (caller falls back to the full
// 136-bit sort).
constexpr int FIX_MAX = 64;

// Byte k of a key (or -1 past its end): packed keys from (hi, lo), long keys
// from their bytes in src at rep's offset.
__device__ __forceinline__ int key_byte_at(u64 h, u64 l, u64 r, const u8* src, u32 k) {
  if (!key_is_long(l)) return k < packed_len(l) ? (int)packed_byte(h, l, k) : -1;
  return k < rep_len(r) ? (int)src[rep_off(r) + k] : -1;
}

// Exact bytewise "a < b" for keys with EQUAL hi (the first 8 bytes).
__device__ __forceinline__ bool tail_less(u64 h, u64 la, u64 ra, u64 lb, u64 rb, const u8* src) {
  if (!key_is_long(la) && !key_is_long(lb)) return la < lb;
  for (u32 k = 8;; ++k) {
    const int x = key_byte_at(h, la, ra, src, k), y = key_byte_at(h, lb, rb, src, k);
    if (x != y) return x < y;  // -1 (end) sorts first: a prefix is smaller
    if (x < 0) return false;
  }
}

__global__ void tie_fixup_kernel(const u64* c, u64* hi, u64* lo, long long* val, u64* rep, u32* part, u64 n,
                                 u32* bad, const u8* src, u64* ln /* optional: key lengths, permuted too */) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    if (i > 0 && c[i] == c[i - 1]) continue;  // not a run head
    u64 e = i + 1;
    while (e < n && c[e] == c[i] && e - i <= (u64)FIX_MAX) ++e;
    if (e - i <= 1) continue;
    if (e - i > (u64)FIX_MAX) {
      atomicOr(bad, 1u);
      continue;
    }
    // insertion sort by exact key order: (hi, lo) for packed keys; with the
    // key bytes (src) also for long keys sharing the 8-byte prefix
    for (u64 a = i + 1; a < e; ++a) {
      const u64 h = hi[a], l = lo[a], r = rep[a];
      const long long v = val[a];
      const u32 p = part[a];
      const u64 k = ln ? ln[a] : 0;
      u64 b = a;
      while (b > i) {
        const u64 hb = hi[b - 1];
        bool greater;
        if (hb != h) greater = hb > h;
        else if (src) greater = tail_less(h, l, r, lo[b - 1], rep[b - 1], src);
        else greater = lo[b - 1] > l;
        if (!greater) break;
        hi[b] = hi[b - 1];
        lo[b] = lo[b - 1];
        val[b] = val[b - 1];
        rep[b] = rep[b - 1];
        part[b] = part[b - 1];
        if (ln) ln[b] = ln[b - 1];
        --b;
      }
      hi[b] = h;
      lo[b] = l;
      val[b] = v;
      rep[b] = r;
      part[b] = p;
      if (ln) ln[b] = k;
    }
    // bit 2 (no key bytes given): two adjacent keys share the 8-byte prefix and
    // one is a long (hashed) key -> the host must check their order bytewise
    if (!src)
      for (u64 a = i + 1; a < e; ++a)
        if (hi[a] == hi[a - 1] && part[a] == part[a - 1] && (key_is_long(lo[a]) || key_is_long(lo[a - 1])))
          atomicOr(bad, 2u);
  }
}

// Gather up to 5 u64 columns and one u32 column by an int32 permutation in
// one launch (the sort's row reorder; replaces one framework gather per column).
__global__ void gather_cols_kernel(const u32* __restrict__ perm, u64 n, const u64* a0, const u64* a1, const u64* a2,
                                   const u64* a3, const u64* a4, const u32* b0, u64* o0, u64* o1, u64* o2, u64* o3,
                                   u64* o4, u32* q0) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const u64 j = clamp_row(perm[i], n);
    if (a0) o0[i] = a0[j];
    if (a1) o1[i] = a1[j];
    if (a2) o2[i] = a2[j];
    if (a3) o3[i] = a3[j];
    if (a4) o4[i] = a4[j];
    if (b0) q0[i] = b0[j];
  }
}

__global__ void composite_key_kernel(const u32* part, const u64* hi, u64 n, u64* out) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    out[i] = ((u64)part[i] << 56) | (hi[i] >> 8);
}

// Device -> pinned-host copy whose length lives in device memory
// (n_bytes = nelem[0] * elem_size, clamped to max_bytes): lets the result
// download be queued without a host synchronisation to learn the size.
// 16-byte stores when both ends are 16-byte aligned; system-scope fence at the
// end so the host sees the data after the stream completes.
// nelem == nullptr: copy exactly max_bytes (size known on the host)
__global__ void copy_to_host_kernel(const u8* src, u8* dst, const long long* nelem, u64 elem_size, u64 max_bytes) {
  u64 nb = nelem ? (u64)nelem[0] * elem_size : max_bytes;
  if (nb > max_bytes) nb = max_bytes;
  const u64 stride = (u64)gridDim.x * blockDim.x;
  const u64 tid = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  const bool vec = (((uintptr_t)src | (uintptr_t)dst) & 15) == 0;
  const u64 nv = vec ? nb / 16 : 0;
  for (u64 i = tid; i < nv; i += stride)
    reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
  for (u64 i = nv * 16 + tid; i < nb; i += stride) dst[i] = src[i];
  // one system-scope release per workgroup, not per thread (a per-thread
  // fence wrote back L2 16 K times per launch and slowed the kernels beside
  // the copy); the host reads only after the stream's completion signal
  __syncthreads();
  if (threadIdx.x == 0) __threadfence_system();
}

}  // namespace mr

using namespace mr;

static inline int grid_n(u64 n, int block, int maxg = 8192) {
  u64 g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > (u64)maxg) g = maxg;
  return (int)g;
}

// single-launch exclusive scan for small arrays (<= 1024 * SS_ITEMS elements):
// each thread keeps its (contiguous) elements in registers — one batch of
// independent loads instead of a serial chain of strided ones (the old form
// read up to 64 elements per thread one after another: 114 us at n = 54k).
constexpr int SS_THREADS = 1024;
constexpr int SS_ITEMS = 16;
template <typename T>
__global__ void __launch_bounds__(SS_THREADS) scan_small_kernel(const T* in, T* out, u64 n, T* total) {
  __shared__ T sh[SS_THREADS / 64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const u64 per = (n + SS_THREADS - 1) / SS_THREADS;  // <= SS_ITEMS
  const u64 b = (u64)t * per;
  T v[SS_ITEMS];
  T s = 0;
#pragma unroll
  for (int k = 0; k < SS_ITEMS; ++k) {
    v[k] = ((u64)k < per && b + k < n) ? in[b + k] : (T)0;
    s += v[k];
  }
  T incl = s;  // wave-inclusive scan of the per-thread sums
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const T y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) sh[wave] = incl;
  __syncthreads();
  T before = 0, all = 0;
#pragma unroll
  for (int w = 0; w < SS_THREADS / 64; ++w) {
    before += w < wave ? sh[w] : (T)0;
    all += sh[w];
  }
  T off = before + incl - s;
#pragma unroll
  for (int k = 0; k < SS_ITEMS; ++k) {
    if ((u64)k < per && b + k < n) out[b + k] = off;
    off += v[k];
  }
  if (t == 0 && total) *total = all;
}

template <typename T>
static int scan_impl(const T* in, T* out, u64 n, T* partials, T* total, hipStream_t s) {
  if (n == 0) return 0;
  if (n <= (u64)SS_THREADS * SS_ITEMS) {
    hipLaunchKernelGGL(scan_small_kernel<T>, dim3(1), dim3(SS_THREADS), 0, s, in, out, n, total);
    return (int)hipGetLastError();
  }
  const u64 nt = (n + SC_TILE - 1) / SC_TILE;
  hipLaunchKernelGGL(scan_reduce_kernel<T>, dim3((unsigned)nt), dim3(SC_THREADS), 0, s, in, n, partials);
  hipLaunchKernelGGL(scan_partials_kernel<T>, dim3(1), dim3(SC_THREADS), 0, s, partials, nt, total);
  hipLaunchKernelGGL(scan_apply_kernel<T>, dim3((unsigned)nt), dim3(SC_THREADS), 0, s, in, n, out, partials);
  return (int)hipGetLastError();
}

template <typename K, int ROUNDS>
static void onesweep_launch(u32 nt, const void* keys_in, const void* vals_in, void* keys_out, void* vals_out, u64 n,
                            int shift, const void* ghist, void* granules, void* tile_counter, u32 epoch, void* err,
                            int iota, int debug_fail, hipStream_t s) {
  hipLaunchKernelGGL((rs_onesweep_kernel<K, u32, ROUNDS>), dim3(nt), dim3(RS_THREADS), 0, s, (const K*)keys_in,
                     (const u32*)vals_in, (K*)keys_out, (u32*)vals_out, n, shift, (const u32*)ghist,
                     (u64*)granules, (u32*)tile_counter, epoch, (u32*)err, iota, debug_fail);
}

template <typename K>
static int onesweep_pass(const void* keys_in, const void* vals_in, void* keys_out, void* vals_out, u64 n, int shift,
                         const void* ghist, void* granules, void* tile_counter, u32 epoch, void* err, int iota,
                         int debug_fail, hipStream_t s);

extern "C" {

u64 mr_scan_partials_len(u64 n) { return (n + SC_TILE - 1) / SC_TILE + 1; }

// The first two launches of the multi-tile exclusive scan: per-tile sums of
// `in` (tiles of mr_scan_tile() items) -> their exclusive scan in partials,
// the total in *total.  A consumer applies partials[tile] itself (the W > 1
// tail: tail.hip's offsets + key-bytes kernel).
u64 mr_scan_tile() { return (u64)SC_TILE; }
int mr_scan_partials_i64(const void* in, u64 n, void* partials, void* total, hipStream_t s) {
  if (n == 0) return 0;
  const u64 nt = (n + SC_TILE - 1) / SC_TILE;
  hipLaunchKernelGGL(scan_reduce_kernel<long long>, dim3((unsigned)nt), dim3(SC_THREADS), 0, s, (const long long*)in,
                     n, (long long*)partials);
  hipLaunchKernelGGL(scan_partials_kernel<long long>, dim3(1), dim3(SC_THREADS), 0, s, (long long*)partials, nt,
                     (long long*)total);
  return (int)hipGetLastError();
}

// exclusive scans; `total` (device, 1 element, may be null) receives the sum
int mr_exclusive_scan_u32(const void* in, void* out, u64 n, void* partials, void* total, hipStream_t s) {
  return scan_impl<u32>((const u32*)in, (u32*)out, n, (u32*)partials, (u32*)total, s);
}
int mr_exclusive_scan_i64(const void* in, void* out, u64 n, void* partials, void* total, hipStream_t s) {
  return scan_impl<long long>((const long long*)in, (long long*)out, n, (long long*)partials, (long long*)total, s);
}

// Global histograms of the digits [d0, ndigits) of a u64 word (ghist: 2048 u32,
// zeroed by caller; digit b at ghist[256 b]).  Flags word: ndigits in bits
// 0-7, MR_GHIST_RUNS (the keys have runs of equal digits), d0 in bits 16-23
// (a sort of the bits >= from_bit needs no histograms below it).
constexpr int MR_GHIST_RUNS = 0x100;
int mr_radix_ghist8(const void* keys, u64 n, void* ghist, int ndigits, hipStream_t s) {
  if (n == 0) return 0;
  const bool runs = (ndigits & MR_GHIST_RUNS) != 0;
  const int d0 = (ndigits >> 16) & 0xFF;
  ndigits &= 0xFF;
  if (runs)
    hipLaunchKernelGGL(rs_ghist8_kernel<true>, dim3(grid_n(n, RS_THREADS, 1024)), dim3(RS_THREADS), 0, s,
                       (const u64*)keys, n, (u32*)ghist, d0, ndigits);
  else
    hipLaunchKernelGGL(rs_ghist8_kernel<false>, dim3(grid_n(n, RS_THREADS, 1024)), dim3(RS_THREADS), 0, s,
                       (const u64*)keys, n, (u32*)ghist, d0, ndigits);
  return (int)hipGetLastError();
}

// One onesweep pass on the 8-bit digit at `shift` (ghist: that digit's 256 bins;
// granules: tiles*256 u64, never needs clearing — entries are epoch tagged;
// tile_counter: one u32 zeroed before the pass; epoch unique per pass).
// granules must hold 256 * mr_onesweep_tiles(n) u64
static int g_onesweep_debug_fail = 0;

// Test knob: the next `passes` onesweep passes (of sorts with at least two
// tiles) give up the look-back of tile 1 — they set the error word and
// scatter with a wrong prefix, as a real give-up would; callers must detect it.
int mr_sort_debug_fail(int passes) {
  g_onesweep_debug_fail = passes;
  return 0;
}

// Rounds (keys per thread) of a onesweep tile (256 threads): 4 up to
// ONESWEEP_SMALL keys, 16 up to ONESWEEP_BIG, `g_big_rounds` above.  Larger
// tiles mean fewer look-back chains and per-tile fixed costs: 100 M keys,
// 0.97 ms per pass at 16 rounds, 0.82 ms at 24 (two workgroups per CU still
// fit in LDS; tools/onesweep_rounds_ab.py, profiles/r2/onesweep/).  Mid-size
// sorts (the word-count tail's ~10^5-10^6 keys) keep 16: there a pass is a
// few tiles' latency, and bigger tiles are fewer and longer.
// u32 keys (the record plane's 32-bit prefixes) take 8 bytes of LDS per key
// with their u32 values instead of 12, so their tiles can be larger: 100 M
// keys, 4 passes, 2.98 ms at 24 rounds, 2.62 at 32 (two workgroups per CU;
// tools/ts_ab.py, profiles/r3/check8/sort_rounds_ab.log).
constexpr u64 ONESWEEP_BIG = 1ull << 22;
static int g_big_rounds = 24;
static int g_big_rounds32 = 32;
int mr_sort_set_rounds(int rounds) {
  if (rounds != 16 && rounds != 24 && rounds != 32) return -1;
  g_big_rounds = rounds;
  return 0;
}
int mr_sort_set_rounds32(int rounds) {
  if (rounds != 16 && rounds != 24 && rounds != 32 && rounds != 40 && rounds != 48) return -1;
  g_big_rounds32 = rounds;
  return 0;
}

// (small sorts: 1024-key tiles; 2048 / 4096 measured slower for the W > 1
// tail's ~10^5 keys, 0.711 / 0.717 vs 0.706 ms per W = 8 proxy step,
// profiles/r5/proxy/)
static int onesweep_rounds(u64 n, int key_bytes) {
  return n <= ONESWEEP_SMALL ? 4 : n < ONESWEEP_BIG ? RS_ROUNDS : (key_bytes == 4 ? g_big_rounds32 : g_big_rounds);
}

static u64 onesweep_tiles_of(u64 n, int key_bytes) {
  const u64 tile = (u64)RS_THREADS * (u64)onesweep_rounds(n, key_bytes);
  return (n + tile - 1) / tile;
}

// look-back granule rows a pass over n keys of either key width may use
u64 mr_onesweep_tiles(u64 n) {
  const u64 a = onesweep_tiles_of(n, 8), b = onesweep_tiles_of(n, 4);
  return a > b ? a : b;
}

}  // extern "C"

template <typename K>
static int onesweep_pass(const void* keys_in, const void* vals_in, void* keys_out, void* vals_out, u64 n, int shift,
                         const void* ghist, void* granules, void* tile_counter, u32 epoch, void* err, int iota,
                         int debug_fail, hipStream_t s) {
  if (n == 0) return 0;
  const u32 nt = (u32)onesweep_tiles_of(n, (int)sizeof(K));
  switch (onesweep_rounds(n, (int)sizeof(K))) {
    case 4: onesweep_launch<K, 4>(nt, keys_in, vals_in, keys_out, vals_out, n, shift, ghist, granules, tile_counter,
                                  epoch, err, iota, debug_fail, s); break;
    case 24: onesweep_launch<K, 24>(nt, keys_in, vals_in, keys_out, vals_out, n, shift, ghist, granules,
                                    tile_counter, epoch, err, iota, debug_fail, s); break;
    case 32: onesweep_launch<K, 32>(nt, keys_in, vals_in, keys_out, vals_out, n, shift, ghist, granules,
                                    tile_counter, epoch, err, iota, debug_fail, s); break;
    case 40:
      if constexpr (sizeof(K) == 4)
        onesweep_launch<K, 40>(nt, keys_in, vals_in, keys_out, vals_out, n, shift, ghist, granules, tile_counter,
                               epoch, err, iota, debug_fail, s);
      break;
    case 48:
      if constexpr (sizeof(K) == 4)
        onesweep_launch<K, 48>(nt, keys_in, vals_in, keys_out, vals_out, n, shift, ghist, granules, tile_counter,
                               epoch, err, iota, debug_fail, s);
      break;
    default: onesweep_launch<K, RS_ROUNDS>(nt, keys_in, vals_in, keys_out, vals_out, n, shift, ghist, granules,
                                           tile_counter, epoch, err, iota, debug_fail, s);
  }
  return (int)hipGetLastError();
}

static int take_debug_fail(u64 n) {
  if (g_onesweep_debug_fail > 0 && mr_onesweep_tiles(n) > 1) {
    --g_onesweep_debug_fail;
    return 1;
  }
  return 0;
}

extern "C" {

int mr_radix_onesweep_u32v(const void* keys_in, const void* vals_in, void* keys_out, void* vals_out, u64 n, int shift,
                           const void* ghist, void* granules, void* tile_counter, u32 epoch, void* err, int iota,
                           hipStream_t s) {
  const int debug_fail = take_debug_fail(n);
  return onesweep_pass<u64>(keys_in, vals_in, keys_out, vals_out, n, shift, ghist, granules, tile_counter, epoch, err,
                            iota, debug_fail, s);
}

// The same pass over u32 keys (shift 0..24).
int mr_radix_onesweep_k32(const void* keys_in, const void* vals_in, void* keys_out, void* vals_out, u64 n, int shift,
                          const void* ghist, void* granules, void* tile_counter, u32 epoch, void* err, int iota,
                          hipStream_t s) {
  const int debug_fail = take_debug_fail(n);
  return onesweep_pass<u32>(keys_in, vals_in, keys_out, vals_out, n, shift, ghist, granules, tile_counter, epoch, err,
                            iota, debug_fail, s);
}

int mr_gather_u64(const void* src, const void* idx, void* dst, u64 n, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(gather_u64_kernel, dim3(grid_n(n, 256)), dim3(256), 0, s, (const u64*)src, (const u32*)idx,
                     (u64*)dst, n);
  return (int)hipGetLastError();
}

int mr_iota_u32(void* dst, u64 n, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(iota_u32_kernel, dim3(grid_n(n, 256)), dim3(256), 0, s, (u32*)dst, n);
  return (int)hipGetLastError();
}

int mr_segment_heads(const void* hi, const void* lo, u64 n, void* heads, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(segment_heads_kernel, dim3(grid_n(n, 256)), dim3(256), 0, s, (const u64*)hi, (const u64*)lo, n,
                     (u32*)heads);
  return (int)hipGetLastError();
}

int mr_segment_fold(const void* seg_excl, const void* heads, const void* vals, u64 n, int op, void* out,
                    hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(segment_fold_kernel, dim3(grid_n(n, 256)), dim3(256), 0, s, (const u32*)seg_excl,
                     (const u32*)heads, (const long long*)vals, n, op, (long long*)out);
  return (int)hipGetLastError();
}

int mr_segment_keys(const void* seg_excl, const void* heads, const void* hi, const void* lo, const void* rep, u64 n,
                    void* out_hi, void* out_lo, void* out_rep, void* out_start, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(segment_keys_kernel, dim3(grid_n(n, 256)), dim3(256), 0, s, (const u32*)seg_excl,
                     (const u32*)heads, (const u64*)hi, (const u64*)lo, (const u64*)rep, n, (u64*)out_hi,
                     (u64*)out_lo, (u64*)out_rep, (u64*)out_start);
  return (int)hipGetLastError();
}

int mr_copy_to_host(const void* src, void* host_dst, const void* nelem, u64 elem_size, u64 max_bytes,
                    hipStream_t s) {
  void* dptr = nullptr;
  if (hipHostGetDevicePointer(&dptr, host_dst, 0) != hipSuccess || dptr == nullptr) dptr = host_dst;
  hipLaunchKernelGGL(copy_to_host_kernel, dim3(1024), dim3(256), 0, s, (const u8*)src, (u8*)dptr,
                     (const long long*)nelem, elem_size, max_bytes);
  return (int)hipGetLastError();
}

// Device -> pinned-host download on stream s (hipMemcpyAsync; this image's
// runtime runs it as a blit kernel).  Shader stores of our own measured slower
// twice: round 1 (0.19 ms on the HBM-resident bench, profiles/r2/d2h_ab/) and
// round 4 on 16-256 workgroups (bigram 26.2-27.9 vs 23.2-23.7 ms,
// profiles/r4/general/bigram_ab/, profiles/r4/rehearse/; profiles/r4/pruned/).
int mr_d2h_async(void* host_dst, const void* src, u64 nbytes, hipStream_t s) {
  if (nbytes == 0) return 0;
  return (int)hipMemcpyAsync(host_dst, src, nbytes, hipMemcpyDeviceToHost, s);
}

// Host-visible completion flags.  A waiting host that sleeps in
// hipStreamSynchronize wakes ~20 us (short waits) to ~130 us (long waits)
// after the GPU work ended (tools/host_gpu_timeline.py); the engine's four
// per-iteration waits instead spin on a word of coherent pinned memory that a
// one-thread kernel queued behind the awaited work stores with release
// semantics at system scope.
__global__ void signal_host_kernel(unsigned int* flag, unsigned int seq) {
  __threadfence_system();
  __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Pinned host memory of exactly `nbytes` (torch's pinned allocator rounds up to
// a power of two, and pinning is paid per page: a 291 MB split buffer cost
// 22 ms as a 512 MB block, inside the cold file-to-result iteration).
void* mr_host_alloc(u64 nbytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, nbytes, hipHostMallocPortable | hipHostMallocMapped) != hipSuccess) return nullptr;
  return p;
}

int mr_host_free(void* p) { return (int)hipHostFree(p); }

void* mr_host_alloc_coherent(u64 nbytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, nbytes, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return nullptr;
  memset(p, 0, nbytes);
  return p;
}

// Small device buffers -> one mapped pinned host buffer, then the host
// flag, in ONE single-workgroup launch (instead of a blit per buffer plus the
// signal kernel: the W > 1 iteration downloads five small tensors at its count
// exchange).  Every thread's stores are vector stores of its own words, each
// followed by a system-scope fence before the barrier; then one lane stores the
// flag with release semantics at system scope.
struct SmallD2H {
  const void* src[8];
  unsigned long long bytes[8];
  unsigned long long off[8];
  int n;
};

__global__ void __launch_bounds__(256) small_d2h_kernel(SmallD2H c, u8* dst, unsigned int* flag, unsigned int seq) {
  for (int j = 0; j < c.n; ++j) {
    const u64 nb = c.bytes[j];
    u8* d = dst + c.off[j];
    if ((nb & 3) == 0) {
      const u32* s = (const u32*)c.src[j];
      for (u64 i = threadIdx.x; i < nb / 4; i += blockDim.x) ((u32*)d)[i] = s[i];
    } else {
      const u8* s = (const u8*)c.src[j];
      for (u64 i = threadIdx.x; i < nb; i += blockDim.x) d[i] = s[i];
    }
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// n (<= 8) device buffers srcs[i] of bytes[i] bytes -> host_dst + offs[i]
// (host_dst: mapped pinned memory, offsets 4-byte aligned), then flag = seq.
int mr_small_d2h(const void* const* srcs, const u64* bytes, const u64* offs, int n, void* host_dst, void* flag_host,
                 unsigned int seq, hipStream_t s) {
  if (n < 0 || n > 8) return -1;
  void* dp = nullptr;
  void* fp = nullptr;
  if (hipHostGetDevicePointer(&dp, host_dst, 0) != hipSuccess || dp == nullptr) return -2;
  if (hipHostGetDevicePointer(&fp, flag_host, 0) != hipSuccess || fp == nullptr) return -2;
  SmallD2H c;
  c.n = n;
  for (int i = 0; i < 8; ++i) {
    c.src[i] = i < n ? srcs[i] : nullptr;
    c.bytes[i] = i < n ? bytes[i] : 0;
    c.off[i] = i < n ? offs[i] : 0;
  }
  hipLaunchKernelGGL(small_d2h_kernel, dim3(1), dim3(256), 0, s, c, (u8*)dp, (unsigned int*)fp, seq);
  return (int)hipGetLastError();
}

int mr_signal_host(void* flag_host, unsigned int seq, hipStream_t s) {
  void* dp = nullptr;
  if (hipHostGetDevicePointer(&dp, flag_host, 0) != hipSuccess || dp == nullptr) return -1;
  hipLaunchKernelGGL(signal_host_kernel, dim3(1), dim3(1), 0, s, (unsigned int*)dp, seq);
  return (int)hipGetLastError();
}

// Host -> device copy by shader loads from pinned host memory (the
// alternative to an SDMA transfer; tools/h2d_probe.py compares them).
__global__ void __launch_bounds__(256) h2d_pull_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                       u64 n16, const u8* __restrict__ src_b, u8* __restrict__ dst_b,
                                                       u64 nbytes) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  const u64 tid = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  u64 i = tid;
  for (; i + 3 * stride < n16; i += 4 * stride) {  // four independent 16-byte loads in flight per thread
    const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n16; i += stride) dst[i] = src[i];
  for (u64 j = n16 * 16 + tid; j < nbytes; j += stride) dst_b[j] = src_b[j];
}

int mr_h2d_pull(void* dst, const void* host_src, u64 nbytes, int blocks, hipStream_t s) {
  if (nbytes == 0) return 0;
  void* sp = nullptr;
  if (hipHostGetDevicePointer(&sp, const_cast<void*>(host_src), 0) != hipSuccess || sp == nullptr)
    sp = const_cast<void*>(host_src);
  if ((((uintptr_t)sp | (uintptr_t)dst) & 15) != 0) return -1;
  hipLaunchKernelGGL(h2d_pull_kernel, dim3(blocks > 0 ? blocks : 2048), dim3(256), 0, s, (const uint4*)sp,
                     (uint4*)dst, nbytes / 16, (const u8*)sp, (u8*)dst, nbytes);
  return (int)hipGetLastError();
}

// Async DMA between pinned host memory and HBM (kind: 1 = H2D, 2 = D2H).
// Used instead of torch's copy_ for the input staging: copy_ also records an
// event for the pinned block in torch's host allocator on every call, and the
// first few of those stalled the host by ~6 ms (tools/first_iter.py).
int mr_memcpy_async(void* dst, const void* src, u64 nbytes, int kind, hipStream_t s) {
  if (nbytes == 0) return 0;
  const hipMemcpyKind k = kind == 1 ? hipMemcpyHostToDevice : (kind == 2 ? hipMemcpyDeviceToHost
                                                                          : hipMemcpyDeviceToDevice);
  return (int)hipMemcpyAsync(dst, src, nbytes, k, s);
}

int mr_composite_key(const void* part, const void* hi, u64 n, void* out, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(composite_key_kernel, dim3(grid_n(n, 256)), dim3(256), 0, s, (const u32*)part, (const u64*)hi,
                     n, (u64*)out);
  return (int)hipGetLastError();
}

int mr_tie_fixup(const void* c, void* hi, void* lo, void* val, void* rep, void* part, u64 n, void* bad,
                 const void* src, void* ln, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(tie_fixup_kernel, dim3(grid_n(n, 256)), dim3(256), 0, s, (const u64*)c, (u64*)hi, (u64*)lo,
                     (long long*)val, (u64*)rep, (u32*)part, n, (u32*)bad, (const u8*)src, (u64*)ln);
  return (int)hipGetLastError();
}

int mr_gather_cols(const void* perm, u64 n, const void* a0, const void* a1, const void* a2, const void* a3,
                   const void* a4, const void* b0, void* o0, void* o1, void* o2, void* o3, void* o4, void* q0,
                   hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(gather_cols_kernel, dim3(grid_n(n, 256)), dim3(256), 0, s, (const u32*)perm, n,
                     (const u64*)a0, (const u64*)a1, (const u64*)a2, (const u64*)a3, (const u64*)a4,
                     (const u32*)b0, (u64*)o0, (u64*)o1, (u64*)o2, (u64*)o3, (u64*)o4, (u32*)q0);
  return (int)hipGetLastError();
}

int mr_bincount(const void* ids, u64 n, u32 nbins, void* counts, hipStream_t s) {
  if (n == 0) return 0;
  if (nbins > 16384) return -1;
  hipLaunchKernelGGL(bincount_kernel, dim3(grid_n(n, 256, 1024)), dim3(256), nbins * sizeof(u32), s,
                     (const u32*)ids, n, nbins, (long long*)counts);
  return (int)hipGetLastError();
}

}  // extern "C"
