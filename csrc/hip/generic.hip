// generic.hip — the general device MapReduce plane (parallel/generic.py):
// arbitrary keys emitted by user device code, folded into typed value columns
// or appended to per-key value lists.
//
// Reference semantics being served (/root/reference/mapreduce/job.lua:83-112):
// ``emit(key, value)`` groups values by key; the reducer (or the combiner taken
// from the reduce module, task.lua:325) folds each key's list.  On the device a
// key is the 128-bit encoding of mr_common.h (exact for <= 15 bytes, prefix +
// hash with byte verification beyond), located in one byte source by its rep
// word; a key maps to a slot of an HBM open-addressing table (hashtab.h,
// OP_NONE: no value in the table itself) and, per slot, either
//   * K typed value columns (i64 / f64 / f32) folded with sum / min / max by
//     native global atomics (gfx950 has global_atomic_{add,min,max}_f64 and
//     add_f32; i64 min/max/add), or
//   * one appended (slot, value) posting per emit (list mode: the reducer
//     sees the whole value list, job.lua:98-106,264-284).
//
// Keys come either pre-encoded (hi, lo, rep) or as byte spans (start, len) of
// a text buffer, packed here in the insert kernel (no intermediate key arrays).
#include <hip/hip_runtime.h>
#include <climits>
#include <cstdlib>
#include "mr_common.h"
#include "hashtab.h"
#include "text_parse.h"

MR_LONG_MASK_SYMBOL(generic)

namespace mr {
namespace ag {

enum VType : int { VT_I64 = 0, VT_F64 = 1, VT_F32 = 2, VT_I32 = 3, VT_SCALAR = 4 };
constexpr int MAXC = 8;

// Column descriptors, passed by value (kernel argument).
struct Cols {
  int k;                       // value columns
  int list;                    // 1: append (slot, value row of the k columns) postings instead of folding
  const void* src[MAXC];       // per-row input values (null for a scalar)
  int stype[MAXC];             // VType of src (VT_SCALAR: the constant sbits, in the dst type)
  long long sbits[MAXC];
  void* dst[MAXC];             // per-slot columns (fold) — or, list mode, dst[0] = posting value rows [n][k]
  int dtype[MAXC];             // VT_I64 / VT_F64 / VT_F32
  int op[MAXC];                // OP_SUM / OP_MIN / OP_MAX
  long long* post_slot;        // list mode: posting slot ids (sink)
  u64 post_base;               // list mode: sink index of row 0
  u32 cs;                      // slot stride of the dst columns in elements (1: one array per
                               // column; 4/8: one row of 8-byte columns per slot, so a key's
                               // folds hit one cache line)
};

struct Keys {
  const u64* hi;
  const u64* lo;
  const u64* rep;
  u64 rep_add;                 // encoded keys: added to rep offsets
  const u8* text;              // spans: key bytes = text[start, start + len)
  const long long* starts;
  const int* lens;
  u64 rep_base;                // spans: rep offset of text[0] in the table's byte source
};

__device__ __forceinline__ long long rd_i64(const Cols& c, int j, u64 i) {
  switch (c.stype[j]) {
    case VT_I64: return ((const long long*)c.src[j])[i];
    case VT_I32: return (long long)((const int*)c.src[j])[i];
    case VT_F64: return (long long)((const double*)c.src[j])[i];
    case VT_F32: return (long long)((const float*)c.src[j])[i];
    default: return c.sbits[j];
  }
}

__device__ __forceinline__ double rd_f64(const Cols& c, int j, u64 i) {
  switch (c.stype[j]) {
    case VT_I64: return (double)((const long long*)c.src[j])[i];
    case VT_I32: return (double)((const int*)c.src[j])[i];
    case VT_F64: return ((const double*)c.src[j])[i];
    case VT_F32: return (double)((const float*)c.src[j])[i];
    default: return __longlong_as_double(c.sbits[j]);
  }
}

__device__ __forceinline__ float rd_f32(const Cols& c, int j, u64 i) {
  switch (c.stype[j]) {
    case VT_I64: return (float)((const long long*)c.src[j])[i];
    case VT_I32: return (float)((const int*)c.src[j])[i];
    case VT_F64: return (float)((const double*)c.src[j])[i];
    case VT_F32: return ((const float*)c.src[j])[i];
    default: return __int_as_float((int)c.sbits[j]);
  }
}

__device__ __forceinline__ void fold_col(const Cols& c, int j, u64 i, u64 slot) {
  const int op = c.op[j];
  if (c.dtype[j] == VT_I64) {
    long long* p = (long long*)c.dst[j] + slot * c.cs;
    const long long v = rd_i64(c, j, i);
    if (op == OP_MIN) atomicMin(p, v);
    else if (op == OP_MAX) atomicMax(p, v);
    else atomicAdd((unsigned long long*)p, (unsigned long long)v);
  } else if (c.dtype[j] == VT_F64) {
    double* p = (double*)c.dst[j] + slot * c.cs;
    const double v = rd_f64(c, j, i);
    if (op == OP_MIN) __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else if (op == OP_MAX) __hip_atomic_fetch_max(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    float* p = (float*)c.dst[j] + slot * c.cs;
    const float v = rd_f32(c, j, i);
    if (op == OP_MIN) __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else if (op == OP_MAX) __hip_atomic_fetch_max(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Little-endian word of the bytes p[0, min(8, avail)) (avail >= 1), the rest
// zero: at most two ALIGNED 8-byte loads, each of a word that holds at least
// one of the wanted bytes (an aligned word never crosses a page, so nothing
// past the buffer's last valid byte's page is touched) — instead of one
// dependent byte load per key byte (profiles/r4/kstats: the span inserts).
__device__ __forceinline__ u64 le_bytes(const u8* p, u64 avail) {
  const uintptr_t a = (uintptr_t)p;
  const u64* w = reinterpret_cast<const u64*>(a & ~(uintptr_t)7);
  const u32 off = (u32)(a & 7);
  u64 x = w[0] >> (8 * off);
  if (off && avail > 8 - off) x |= w[1] << (64 - 8 * off);
  if (avail < 8) x &= (1ull << (8 * avail)) - 1;
  return x;
}

// 128-bit key of text[s, s + len) (mr_common.h encoding; len >= 1).
__device__ __forceinline__ void span_key(const u8* text, u64 s, u64 len, u64& hi, u64& lo) {
  const u8* p = text + s;
  hi = __builtin_bswap64(le_bytes(p, len));
  if (len <= (u64)PACK_MAX) {
    lo = (len > 8 ? __builtin_bswap64(le_bytes(p + 8, len - 8)) : 0ull) | len;
    return;
  }
  u64 h = long_hash_init(len);
  for (u64 w = 0; w < len; w += 8) h = long_hash_step(h, le_bytes(p + w, len - w));
  lo = long_lo(h, mr_long_mask);
}

// One row per thread: key -> slot (insert or find), then fold the row's values
// into the slot's columns, or append its posting.  Rows with an empty span
// (len <= 0) are skipped (list mode: posting slot -1).  An insert that runs
// out of probes sets the table's overflow flag; the host regrows and re-runs.
__global__ void __launch_bounds__(256) agg_insert_kernel(GTab g, Keys ks, u64 n, Cols c) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  u32 claims = 0;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    u64 hi = 0, lo = 0, rep = 0;
    bool ok = true;
    if (ks.text) {
      const long long s = ks.starts[i];
      const int len = ks.lens[i];
      if (len <= 0 || s < 0) {
        ok = false;
      } else {
        span_key(ks.text, (u64)s, (u64)len, hi, lo);
        rep = make_rep(ks.rep_base + (u64)s, (u64)len);
      }
    } else {
      hi = ks.hi[i];
      lo = ks.lo[i];
      rep = ks.rep ? ks.rep[i] + (ks.rep_add << REP_LEN_BITS) : 0;
    }
    u64 slot = 0;
    int r = 0;
    if (ok) {
      r = gtab_insert(g, hi, lo, 0, rep, OP_NONE, &slot);
      claims += r == 2;
    }
    if (c.list) {
      // a posting = the key's slot + a value row of k 8-byte words (int64 /
      // float64 bits; byte-string values are span words of the byte source)
      c.post_slot[c.post_base + i] = r ? (long long)slot : -1;
      long long* row = (long long*)c.dst[0] + (c.post_base + i) * (u64)c.k;
      for (int j = 0; j < c.k; ++j)
        row[j] = c.dtype[j] == VT_F64 ? __double_as_longlong(rd_f64(c, j, i)) : rd_i64(c, j, i);
    } else if (r) {
      for (int j = 0; j < c.k; ++j) fold_col(c, j, i, slot);
    }
  }
  gtab_count_claims(g, claims);
}

// Occupied slots -> dense (slot, hi, lo, rep), in slot order: slots ranked
// k-major inside the block (b0 + k*256 + t), so the lanes of a wave write
// consecutive rows for each k (ballot + popcount per (k, wave), a 64-entry
// scan in LDS, one atomic per block for its base).
constexpr int SC_ITEMS = 16;
__global__ void __launch_bounds__(256) slot_compact_kernel(GTab g, u64 cap, long long* out_slot, u64* out_hi,
                                                           u64* out_lo, u64* out_rep, unsigned long long* counter) {
  constexpr int NW = 256 / 64;
  __shared__ u32 wc[SC_ITEMS * NW];
  __shared__ unsigned long long base;
  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  const unsigned long long below = (1ull << lane) - 1ull;
  const u64 b0 = (u64)blockIdx.x * 256 * SC_ITEMS;
  u32 occ = 0;
  u32 rank[SC_ITEMS];
#pragma unroll
  for (int k = 0; k < SC_ITEMS; ++k) {
    const u64 i = b0 + (u64)k * 256 + t;
    const bool o = i < cap && g.s[i].tag != 0;
    occ |= (o ? 1u : 0u) << k;
    const unsigned long long m = __ballot(o);
    rank[k] = (u32)__popcll(m & below);
    if (lane == 0) wc[k * NW + wave] = (u32)__popcll(m);
  }
  __syncthreads();
  if (t < 64) {
    const u32 c = t < SC_ITEMS * NW ? wc[t] : 0u;
    u32 incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const u32 v = __shfl_up(incl, o);
      if (lane >= o) incl += v;
    }
    if (t < SC_ITEMS * NW) wc[t] = incl - c;
    if (t == 63) base = atomicAdd(counter, (unsigned long long)incl);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < SC_ITEMS; ++k) {
    if (occ & (1u << k)) {
      const u64 i = b0 + (u64)k * 256 + t;
      const u64 o = base + wc[k * NW + wave] + rank[k];
      out_slot[o] = (long long)i;
      out_hi[o] = g.s[i].hi;
      out_lo[o] = g.s[i].lo;
      out_rep[o] = g.s[i].rep;
    }
  }
}

// ---------------------------------------------------------------------------
// Fold mode with an LDS combine (skewed keys: a Zipf-hot key would otherwise
// take one memory-side atomic per row, all on the same address).  A block
// takes CB_ROWS consecutive rows: keys of <= 15 bytes are combined in a
// CB_SLOTS-slot LDS table whose per-slot partial columns are folded with LDS
// atomics (f32 columns accumulate in f64); the block then inserts each of its
// distinct keys into the HBM table once and folds the partials with one
// global atomic per column.  Long keys (prefix + hash, verified by bytes in
// the global table) and rows past the LDS table's load limit take the direct
// per-row path of agg_insert_kernel.
// 512 threads per block: with 4 value columns the block's LDS (64 KiB) allows
// two blocks per CU, and 16 waves hide the per-row load chains better than 8
// (CSV group-by 5.49 -> 5.13 ms per step, bigram unchanged;
// profiles/r3/check7/generic_combine_block_ab.txt).
constexpr int CB_T = 512, CB_ROWS = 4096, CB_SLOTS = 1024;
constexpr int CB_LIMIT = CB_SLOTS * 3 / 4, CB_PROBES = 32;

__device__ __forceinline__ long long cb_identity(int dtype, int op) {
  if (dtype == VT_I64) return op == OP_MIN ? LLONG_MAX : (op == OP_MAX ? LLONG_MIN : 0ll);
  return __double_as_longlong(op == OP_MIN ? __builtin_inf() : (op == OP_MAX ? -__builtin_inf() : 0.0));
}

__device__ __forceinline__ void cb_lds_fold(long long* acc, const Cols& c, int j, u64 i) {
  const int op = c.op[j];
  if (c.dtype[j] == VT_I64) {
    const long long v = rd_i64(c, j, i);
    if (op == OP_MIN) atomicMin(acc, v);
    else if (op == OP_MAX) atomicMax(acc, v);
    else atomicAdd((unsigned long long*)acc, (unsigned long long)v);
  } else {
    double* p = (double*)acc;
    const double v = c.dtype[j] == VT_F64 ? rd_f64(c, j, i) : (double)rd_f32(c, j, i);
    if (op == OP_MIN) __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else if (op == OP_MAX) __hip_atomic_fetch_max(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

// One block partial (bits in the LDS accumulator's representation) into slot.
__device__ __forceinline__ void cb_global_fold(const Cols& c, int j, u64 slot, long long bits) {
  const int op = c.op[j];
  if (c.dtype[j] == VT_I64) {
    long long* p = (long long*)c.dst[j] + slot * c.cs;
    if (op == OP_MIN) atomicMin(p, bits);
    else if (op == OP_MAX) atomicMax(p, bits);
    else atomicAdd((unsigned long long*)p, (unsigned long long)bits);
  } else if (c.dtype[j] == VT_F64) {
    double* p = (double*)c.dst[j] + slot * c.cs;
    const double v = __longlong_as_double(bits);
    if (op == OP_MIN) __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else if (op == OP_MAX) __hip_atomic_fetch_max(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    float* p = (float*)c.dst[j] + slot * c.cs;
    const float v = (float)__longlong_as_double(bits);
    if (op == OP_MIN) __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else if (op == OP_MAX) __hip_atomic_fetch_max(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// LDS slot of a packed key (claimed if absent), or -1 (table at its limit).
// A key of <= 7 bytes is its own tag (one LDS read on a hit); longer packed
// keys use a hashed tag plus the (hi, lo) published by the claimer (lo last).
__device__ __forceinline__ int cb_slot(u64* tag, u64* khi, u64* klo, u64* krep, u32* nclaimed, u64 hi, u64 lo,
                                       u64 rep) {
  u64 h = hi ^ (lo * 0x9E3779B97F4A7C15ull);
  h ^= h >> 31;
  h *= 0xC2B2AE3D27D4EB4Full;
  h ^= h >> 29;
  const bool exact = (lo - 1 < 7) && (hi & 0xFFull) == 0;
  const u64 t = exact ? (hi | lo) : ((h & ~0xFFull) | 0x80ull);
  u32 s = (u32)(h >> 40) & (CB_SLOTS - 1);
  for (int probes = 0; probes < CB_PROBES;) {
    u64 cur = __hip_atomic_load(&tag[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (cur == 0) {
      if (__hip_atomic_load(nclaimed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= (u32)CB_LIMIT) return -1;
      u64 expected = 0;
      if (__hip_atomic_compare_exchange_strong(&tag[s], &expected, t, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP)) {
        khi[s] = hi;
        krep[s] = rep;
        __hip_atomic_fetch_add(nclaimed, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_store(&klo[s], lo, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        return (int)s;
      }
      cur = expected;
    }
    if (cur == t) {
      if (exact) return (int)s;
      const u64 l = __hip_atomic_load(&klo[s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (l == 0) continue;  // the claimer has not published yet: re-read this slot
      if (l == lo && khi[s] == hi) return (int)s;
    }
    s = (s + 1) & (CB_SLOTS - 1);
    ++probes;
  }
  return -1;
}

// The keys of a thread's rows r0 + it * CB_T + threadIdx.x (it < items), their
// loads issued together (span starts/lengths, then the key words: independent
// chains, so the row loop after it does not wait a memory round trip per
// row); returns the mask of rows with a key.
template <int ITEMS, int STRIDE = CB_T>
__device__ __forceinline__ u32 cb_row_keys(const Keys& ks, u64 r0, int items, u64 n, u64 (&khi_r)[ITEMS],
                                           u64 (&klo_r)[ITEMS], u64 (&krep_r)[ITEMS]) {
  const int t = threadIdx.x;
  u32 ok = 0;
  if (ks.text) {
    long long st_r[ITEMS];
    int len_r[ITEMS];
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
      const u64 i = r0 + (u64)it * STRIDE + t;
      const bool in = it < items && i < n;
      st_r[it] = in ? ks.starts[i] : -1;
      len_r[it] = in ? ks.lens[i] : 0;
    }
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
      khi_r[it] = klo_r[it] = krep_r[it] = 0;
      if (len_r[it] > 0 && st_r[it] >= 0) {
        span_key(ks.text, (u64)st_r[it], (u64)len_r[it], khi_r[it], klo_r[it]);
        krep_r[it] = make_rep(ks.rep_base + (u64)st_r[it], (u64)len_r[it]);
        ok |= 1u << it;
      }
    }
  } else {
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
      const u64 i = r0 + (u64)it * STRIDE + t;
      const bool in = it < items && i < n;
      khi_r[it] = in ? ks.hi[i] : 0;
      klo_r[it] = in ? ks.lo[i] : 0;
      krep_r[it] = (in && ks.rep) ? ks.rep[i] + (ks.rep_add << REP_LEN_BITS) : 0;
      if (in) ok |= 1u << it;
    }
  }
  return ok;
}

// rows: rows per block (a multiple of CB_T, at most CB_ROWS): small batches get
// smaller blocks so the launch still covers the chip (a 2-8 MiB CSV chunk at
// 4096 rows per block ran 37-150 blocks on 256 CUs, 72 % of wave cycles
// waiting: profiles/r4/general/csv_pmc/)
// BATCH (mr_agg_set_batch): the rows that go to the HBM table directly, and
// the flush of the LDS-combined keys, probe their home slots in batches
// (gtab_find_or_claim_home) instead of one gtab_insert per key.
template <bool BATCH, int PH>
__global__ void __launch_bounds__(CB_T) agg_combine_kernel(GTab g, Keys ks, u64 n, Cols c, u32 rows) {
  constexpr int CB_ITEMS = CB_ROWS / CB_T;
  const int items = (int)(rows / CB_T);
  extern __shared__ __attribute__((aligned(16))) u64 lds[];
  u64* tag = lds;
  u64* khi = tag + CB_SLOTS;
  u64* klo = khi + CB_SLOTS;
  u64* krep = klo + CB_SLOTS;
  long long* acc = (long long*)(krep + CB_SLOTS);  // [c.k][CB_SLOTS]
  __shared__ u32 nclaimed;
  const int t = threadIdx.x;
  for (int s = t; s < CB_SLOTS; s += CB_T) {
    tag[s] = 0;
    klo[s] = 0;
    for (int j = 0; j < c.k; ++j) acc[j * CB_SLOTS + s] = cb_identity(c.dtype[j], c.op[j]);
  }
  if (t == 0) nclaimed = 0;
  __syncthreads();
  u32 claims = 0;
  const u64 r0 = (u64)blockIdx.x * rows;
  // rows whose key found no room in the LDS table (or is long) go to the HBM
  // table directly — BATCH: all of a thread's such rows probe their home
  // slots together (gtab_find_or_claim_home), the rest one by one.  With few
  // repeats inside a block (bigrams: 23 M distinct of 47 M) that is most rows,
  // and one dependent claim chain per row had kept 82 % of the wave cycles
  // waiting (profiles/r5/bigram/pmc/).
  if constexpr (!BATCH && PH > 1) {
    // PH phases of CB_ITEMS / PH rows per thread: PH = 2 holds half the row
    // keys in registers (56 VGPRs: 7 waves per SIMD instead of 6)
    constexpr int HI = CB_ITEMS / PH;
#pragma unroll
    for (int ph = 0; ph < PH; ++ph) {
      u64 khi_r[HI], klo_r[HI], krep_r[HI];
      const u64 rb = r0 + (u64)ph * HI * CB_T;
      const u32 ok = cb_row_keys<HI>(ks, rb, items - ph * HI, n, khi_r, klo_r, krep_r);
#pragma unroll
      for (int it = 0; it < HI; ++it) {
        const u64 i = rb + (u64)it * CB_T + t;
        if (!(ok & (1u << it))) continue;
        const u64 hi = khi_r[it], lo = klo_r[it], rep = krep_r[it];
        const int s = key_is_long(lo) ? -1 : cb_slot(tag, khi, klo, krep, &nclaimed, hi, lo, rep);
        if (s >= 0) {
          for (int j = 0; j < c.k; ++j) cb_lds_fold(&acc[j * CB_SLOTS + s], c, j, i);
        } else {
          u64 slot = 0;
          const int r = gtab_insert(g, hi, lo, 0, rep, OP_NONE, &slot);
          claims += r == 2;
          if (r)
            for (int j = 0; j < c.k; ++j) fold_col(c, j, i, slot);
        }
      }
    }
  } else {
    u64 khi_r[CB_ITEMS], klo_r[CB_ITEMS], krep_r[CB_ITEMS];
    const u32 ok = cb_row_keys<CB_ITEMS>(ks, r0, items, n, khi_r, klo_r, krep_r);
    u32 direct = 0;
#pragma unroll
    for (int it = 0; it < CB_ITEMS; ++it) {
      const u64 i = r0 + (u64)it * CB_T + t;
      if (!(ok & (1u << it))) continue;
      const u64 hi = khi_r[it], lo = klo_r[it], rep = krep_r[it];
      const int s = key_is_long(lo) ? -1 : cb_slot(tag, khi, klo, krep, &nclaimed, hi, lo, rep);
      if (s >= 0) {
        for (int j = 0; j < c.k; ++j) cb_lds_fold(&acc[j * CB_SLOTS + s], c, j, i);
      } else if constexpr (BATCH) {
        direct |= 1u << it;
      } else {
        u64 slot = 0;
        const int r = gtab_insert(g, hi, lo, 0, rep, OP_NONE, &slot);
        claims += r == 2;
        if (r)
          for (int j = 0; j < c.k; ++j) fold_col(c, j, i, slot);
      }
    }
    if (BATCH && direct) {
      u64 dslot[CB_ITEMS];
      u32 won = 0, w2 = 0;
      static_assert(CB_ITEMS == 8, "two batches of four");
      u32 done = gtab_find_or_claim_home<4, 0>(g, khi_r, klo_r, krep_r, direct, dslot, won);
      done |= gtab_find_or_claim_home<4, 4>(g, khi_r, klo_r, krep_r, direct, dslot, w2);
      claims += __builtin_popcount(won | w2);
#pragma unroll
      for (int it = 0; it < CB_ITEMS; ++it) {
        if (!(direct & (1u << it))) continue;
        const u64 i = r0 + (u64)it * CB_T + t;
        u64 slot = dslot[it];
        int r = 1;
        if (!(done & (1u << it))) {
          r = gtab_insert(g, khi_r[it], klo_r[it], 0, krep_r[it], OP_NONE, &slot);
          claims += r == 2;
        }
        if (r)
          for (int j = 0; j < c.k; ++j) fold_col(c, j, i, slot);
      }
    }
  }
  __syncthreads();
  if constexpr (!BATCH) {
    for (int s = t; s < CB_SLOTS; s += CB_T) {
      if (!tag[s]) continue;
      u64 slot = 0;
      const int r = gtab_insert(g, khi[s], klo[s], 0, krep[s], OP_NONE, &slot);
      claims += r == 2;
      if (r)
        for (int j = 0; j < c.k; ++j) cb_global_fold(c, j, slot, acc[j * CB_SLOTS + s]);
    }
    gtab_count_claims(g, claims);
    return;
  }
  // the block's LDS-combined keys: the same batched probe, 2 per thread
  constexpr int PER = CB_SLOTS / CB_T;
  u64 fhi[PER], flo[PER], frep[PER], fslot[PER];
  u32 occ = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int s = t + k * CB_T;
    fhi[k] = khi[s];
    flo[k] = klo[s];
    frep[k] = krep[s];
    if (tag[s]) occ |= 1u << k;
  }
  if (occ) {
    u32 won = 0;
    const u32 done = gtab_find_or_claim_home<PER, 0>(g, fhi, flo, frep, occ, fslot, won);
    claims += __builtin_popcount(won);
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      if (!(occ & (1u << k))) continue;
      const int s = t + k * CB_T;
      u64 slot = fslot[k];
      int r = 1;
      if (!(done & (1u << k))) {
        r = gtab_insert(g, fhi[k], flo[k], 0, frep[k], OP_NONE, &slot);
        claims += r == 2;
      }
      if (r)
        for (int j = 0; j < c.k; ++j) cb_global_fold(c, j, slot, acc[j * CB_SLOTS + s]);
    }
  }
  gtab_count_claims(g, claims);
}

// ---------------------------------------------------------------------------
// Fused CSV fold (emit.csv): lines -> fields -> decimal parse -> LDS combine
// -> HBM table, in one kernel that reads the text once — instead of the op
// chain lines / field / field / parse / mask / insert (six launches and five
// intermediate arrays per chunk).  Line and field rules are text.hip's
// (ops/text.py is the specification): a line starts at byte 0 or after a
// '\n'; a trailing '\r' is not part of the line's last field; a missing key
// or value field, an empty key, or a value that does not parse drops the row.
// Each block takes `tiles` consecutive 8 KiB tiles: per tile the line starts
// are found from a newline mask of 16 bytes per thread and compacted by a
// block scan, then processed lane per line; a line belongs to the tile of
// its first byte (its bytes past the tile are read from global memory).
constexpr int CV_SEG = 16, CV_TILE = CB_T * CV_SEG;  // 8 KiB tiles, 512 threads
constexpr int CV_MAXV = 4;                          // value inputs of a fused CSV fold

// the value of input i (0..3) among four registers (no register-array indexing)
__device__ __forceinline__ double pick(double v0, double v1, double v2, double v3, int i) {
  return i == 0 ? v0 : (i == 1 ? v1 : (i == 2 ? v2 : v3));
}

struct CsvSpec {
  int sep;
  int kf;              // key field
  int nin;             // input (value) columns
  int vf[MAXC];        // per input column: its field, or -1 = the constant 1
  int pin[MAXC];       // per physical column: its input column, or -1 = the scalar c.sbits
};

__device__ __forceinline__ double scalar_of(const Cols& c, int j) {
  return c.dtype[j] == VT_I64 ? (double)c.sbits[j] : __longlong_as_double(c.sbits[j]);
}

__device__ __forceinline__ void cv_lds_fold(long long* acc, int dtype, int op, double v) {
  if (dtype == VT_I64) {
    const long long x = (long long)v;
    if (op == OP_MIN) atomicMin(acc, x);
    else if (op == OP_MAX) atomicMax(acc, x);
    else atomicAdd((unsigned long long*)acc, (unsigned long long)x);
  } else {
    double* p = (double*)acc;
    const double x = dtype == VT_F32 ? (double)(float)v : v;
    if (op == OP_MIN) __hip_atomic_fetch_min(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else if (op == OP_MAX) __hip_atomic_fetch_max(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else __hip_atomic_fetch_add(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

__device__ __forceinline__ void cv_global_fold(const Cols& c, int j, u64 slot, double v) {
  const int op = c.op[j];
  if (c.dtype[j] == VT_I64) {
    long long* p = (long long*)c.dst[j] + slot * c.cs;
    const long long x = (long long)v;
    if (op == OP_MIN) atomicMin(p, x);
    else if (op == OP_MAX) atomicMax(p, x);
    else atomicAdd((unsigned long long*)p, (unsigned long long)x);
  } else if (c.dtype[j] == VT_F64) {
    double* p = (double*)c.dst[j] + slot * c.cs;
    if (op == OP_MIN) __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else if (op == OP_MAX) __hip_atomic_fetch_max(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    float* p = (float*)c.dst[j] + slot * c.cs;
    const float x = (float)v;
    if (op == OP_MIN) __hip_atomic_fetch_min(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else if (op == OP_MAX) __hip_atomic_fetch_max(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else __hip_atomic_fetch_add(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// First set bit of a tile bit mask (1 bit per byte, u32 words) at a position
// in [from, to), or `to`.
__device__ __forceinline__ u32 cv_next_bit(const u32* w, u32 from, u32 to) {
  u32 i = from;
  while (i < to) {
    const u32 m = w[i >> 5] >> (i & 31);
    if (m) {
      const u32 p = i + (u32)__builtin_ctz(m);
      return p < to ? p : to;
    }
    i = (i | 31) + 1;
  }
  return to;
}

constexpr int CV_LP = 4096;  // line starts ranked per pass (a tile of shorter lines takes two passes)

__global__ void __launch_bounds__(CB_T) __attribute__((amdgpu_waves_per_eu(4, 8)))
csv_fold_kernel(GTab g, const u8* __restrict__ text, u64 n, u64 rep_base, CsvSpec sp, Cols c, u32 tiles,
                unsigned long long* __restrict__ rows_out, int mode) {
  extern __shared__ __attribute__((aligned(16))) u64 lds[];
  u64* tag = lds;
  u64* khi = tag + CB_SLOTS;
  u64* klo = khi + CB_SLOTS;
  u64* krep = klo + CB_SLOTS;
  long long* acc = (long long*)(krep + CB_SLOTS);  // [c.k][CB_SLOTS]
  // the tile's bytes and its newline / separator bit masks: the per-line walks
  // below read LDS (a byte-serial walk through global memory was latency-bound)
  __shared__ __attribute__((aligned(16))) u64 tb64[CV_TILE / 8 + 2];
  __shared__ u32 nlw[CV_TILE / 32 + 1], spw[CV_TILE / 32 + 1];
  __shared__ u16 lpos[CV_LP];
  __shared__ u32 wsum[CB_T / 64];
  __shared__ u32 nclaimed, nrows;
  const u8* tb = (const u8*)tb64;
  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  for (int q = t; q < CB_SLOTS; q += CB_T) {
    tag[q] = 0;
    klo[q] = 0;
    for (int j = 0; j < c.k; ++j) acc[j * CB_SLOTS + q] = cb_identity(c.dtype[j], c.op[j]);
  }
  if (t == 0) {
    nclaimed = nrows = 0;
    nlw[CV_TILE / 32] = spw[CV_TILE / 32] = 0;
    tb64[CV_TILE / 8] = tb64[CV_TILE / 8 + 1] = 0;
  }
  int maxf = sp.kf;
#pragma unroll
  for (int j = 0; j < CV_MAXV; ++j)
    if (j < sp.nin && sp.vf[j] > maxf) maxf = sp.vf[j];
  u32 need = 0;  // inputs read from a field
#pragma unroll
  for (int j = 0; j < CV_MAXV; ++j)
    if (j < sp.nin && sp.vf[j] >= 0) need |= 1u << j;
  const u8 sep = (u8)sp.sep;
  __syncthreads();
  u32 claims = 0, myrows = 0;
  const u64 b0 = (u64)blockIdx.x * tiles * (u64)CV_TILE;
  for (u32 tt = 0; tt < tiles; ++tt) {
    const u64 tile = b0 + (u64)tt * CV_TILE;
    if (tile >= n) break;  // (uniform across the block)
    const u64 tend = n - tile < (u64)CV_TILE ? n : tile + CV_TILE;  // bytes [tile, tend) are in LDS
    const u32 tlen = (u32)(tend - tile);
    const u64 gpos = tile + (u64)t * CV_SEG;
    u32 starts = 0, nlm = 0, spm = 0;
    uint4 q = make_uint4(0u, 0u, 0u, 0u);
    if (gpos + CV_SEG <= n && (((uintptr_t)(text + gpos)) & 15) == 0) {
      q = *reinterpret_cast<const uint4*>(text + gpos);
    } else if (gpos < n) {
      u32 w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int i = 0; i < CV_SEG; ++i)
        if (gpos + i < n) w[i >> 2] |= (u32)text[gpos + i] << (8 * (i & 3));
      q = make_uint4(w[0], w[1], w[2], w[3]);
    }
    reinterpret_cast<uint4*>(tb64)[t] = q;
    {
      const u32 w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int i = 0; i < CV_SEG; ++i) {
        const u32 ch = (w[i >> 2] >> (8 * (i & 3))) & 0xFFu;
        nlm |= (ch == 10u ? 1u : 0u) << i;
        spm |= (ch == (u32)sep ? 1u : 0u) << i;
      }
    }
    if (gpos < n) {
      const u32 prev = (gpos == 0 || text[gpos - 1] == 10) ? 1u : 0u;
      starts = ((nlm << 1) | prev) & 0xFFFFu;
      const u64 lim = n - gpos;
      if (lim < (u64)CV_SEG) {
        const u32 keep = (1u << lim) - 1u;
        starts &= keep;
        nlm &= keep;
        spm &= keep;
      }
    }
    reinterpret_cast<u16*>(nlw)[t] = (u16)nlm;
    reinterpret_cast<u16*>(spw)[t] = (u16)spm;
    // block exclusive scan of the line-start counts
    const u32 cnt = (u32)__builtin_popcount(starts);
    u32 incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const u32 v = __shfl_up(incl, o);
      if (lane >= o) incl += v;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    u32 base = 0, total = 0;
#pragma unroll
    for (int w = 0; w < CB_T / 64; ++w) {
      const u32 x = wsum[w];
      base += w < wave ? x : 0u;
      total += x;
    }
    const u32 kx = base + incl - cnt;
    for (u32 p0 = 0; p0 < total; p0 += CV_LP) {  // (uniform)
      {
        u32 k = kx, st = starts;
        while (st) {
          const int i = __builtin_ctz(st);
          st &= st - 1;
          if (k >= p0 && k < p0 + CV_LP) lpos[k - p0] = (u16)(t * CV_SEG + i);
          ++k;
        }
      }
      __syncthreads();
      const u32 cntp = total - p0 < (u32)CV_LP ? total - p0 : (u32)CV_LP;
      for (u32 x = t; x < cntp; x += CB_T) {
        const u32 rs = lpos[x];  // tile offset of the line start
        // line end: the next newline (LDS mask), past the tile through global memory
        u32 re = cv_next_bit(nlw, rs, tlen);
        u64 le = tile + re;
        if (re == tlen) {
          while (le < n && text[le] != 10) ++le;
        }
        if (le > tile + rs) {
          const u64 l1 = le - 1;
          if ((l1 < tend ? tb[l1 - tile] : text[l1]) == 13) --le;
        }
        int klen = -1;
        u64 ks = 0;
        double v0 = 1.0, v1 = 1.0, v2 = 1.0, v3 = 1.0;  // inputs without a field stay 1
        u32 got = 0;
        bool bad = false;
        u64 fs = tile + rs;
        for (int f = 0; f <= maxf; ++f) {
          // the field's end: the next separator before the line end
          const u64 lim = le < tend ? le : tend;
          u64 fe;
          if (fs < lim) {
            fe = tile + cv_next_bit(spw, (u32)(fs - tile), (u32)(lim - tile));
          } else {
            fe = fs;
          }
          if (fe >= lim && fe < le) {  // the field runs past the tile
            while (fe < le && text[fe] != sep) ++fe;
          }
          const int flen = (int)(fe - fs);
          if (f == sp.kf) {
            ks = fs;
            klen = flen;
          }
          u32 hit = 0;
#pragma unroll
          for (int j = 0; j < CV_MAXV; ++j) hit |= (j < sp.nin && sp.vf[j] == f ? 1u : 0u) << j;
          if (hit) {
            bool b = false;
            const double v = fe <= tend ? tx::parse_f64(tb + (fs - tile), flen, b) : tx::parse_f64(text + fs, flen, b);
            bad |= b;
            got |= hit;
            if (hit & 1u) v0 = v;
            if (hit & 2u) v1 = v;
            if (hit & 4u) v2 = v;
            if (hit & 8u) v3 = v;
          }
          if (fe >= le) break;
          fs = fe + 1;
        }
        if (bad || klen <= 0 || (got & need) != need) continue;
        ++myrows;
        if (mode == 1) continue;  // (ablation: parse only)
        u64 hi, lo;
        if (ks + (u64)klen <= tend) span_key(tb, ks - tile, (u64)klen, hi, lo);
        else span_key(text, ks, (u64)klen, hi, lo);
        const u64 rep = make_rep(rep_base + ks, (u64)klen);
        const int sl = (key_is_long(lo) || mode == 2) ? -1 : cb_slot(tag, khi, klo, krep, &nclaimed, hi, lo, rep);
        if (sl >= 0) {
          for (int j = 0; j < c.k; ++j) {
            const int i = sp.pin[j];
            const double v = i >= 0 ? pick(v0, v1, v2, v3, i) : scalar_of(c, j);
            cv_lds_fold(&acc[j * CB_SLOTS + sl], c.dtype[j], c.op[j], v);
          }
        } else {
          u64 slot = 0;
          const int r = gtab_insert(g, hi, lo, 0, rep, OP_NONE, &slot);
          claims += r == 2;
          if (r)
            for (int j = 0; j < c.k; ++j) {
              const int i = sp.pin[j];
              const double v = i >= 0 ? pick(v0, v1, v2, v3, i) : scalar_of(c, j);
              cv_global_fold(c, j, slot, v);
            }
        }
      }
      __syncthreads();
    }
    __syncthreads();  // (a tile without line starts: wsum and the LDS tile are rewritten next)
  }
  if (myrows) atomicAdd(&nrows, myrows);
  __syncthreads();
  if (t == 0 && nrows) atomicAdd(rows_out, (unsigned long long)nrows);
  for (int s = t; s < CB_SLOTS; s += CB_T) {
    if (!tag[s]) continue;
    u64 slot = 0;
    const int r = gtab_insert(g, khi[s], klo[s], 0, krep[s], OP_NONE, &slot);
    claims += r == 2;
    if (r)
      for (int j = 0; j < c.k; ++j) cb_global_fold(c, j, slot, acc[j * CB_SLOTS + s]);
  }
  gtab_count_claims(g, claims);
}

// Fill a typed column with its fold identity (sum 0, min +max, max -max).
__global__ void col_fill_kernel(void* col, u64 n, long long bits, int width) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    if (width == 8) ((long long*)col)[i] = bits;
    else ((int*)col)[i] = (int)bits;
  }
}

}  // namespace ag
}  // namespace mr

using namespace mr;
using namespace mr::ag;

static inline unsigned ag_grid(u64 n, unsigned block, unsigned cap = 8192) {
  u64 g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

static inline GTab ag_gtab(void* tag, void* hi, void* lo, void* val, void* rep, void* ctrl, u64 cap, const void* src) {
  GTab g = gtab_make(tag, val, ctrl, cap, (const u8*)src);
  return g;
}

// Host-side mirror of Cols for ctypes (same field order, fixed arrays).
struct ColsArg {
  long long k, list;
  const void* src[MAXC];
  long long stype[MAXC];
  long long sbits[MAXC];
  void* dst[MAXC];
  long long dtype[MAXC];
  long long op[MAXC];
  void* post_slot;
  unsigned long long post_base;
  long long rows_only;  // 1: one row per thread (distinct keys: an LDS combine has nothing to fold)
  long long cstride;    // slot stride of the dst columns (elements; 0 = 1)
};

static Cols to_cols(const ColsArg* a) {
  Cols c;
  c.k = (int)a->k;
  c.list = (int)a->list;
  for (int j = 0; j < MAXC; ++j) {
    c.src[j] = a->src[j];
    c.stype[j] = (int)a->stype[j];
    c.sbits[j] = a->sbits[j];
    c.dst[j] = a->dst[j];
    c.dtype[j] = (int)a->dtype[j];
    c.op[j] = (int)a->op[j];
  }
  c.post_slot = (long long*)a->post_slot;
  c.post_base = a->post_base;
  c.cs = a->cstride > 0 ? (u32)a->cstride : 1u;
  return c;
}

// workgroup cap of the per-row insert: one row per thread up to 16 M rows
// (the insert is probe-latency-bound; 65536 vs 8192 vs 2048 workgroups:
// reducefn3 6.57-6.62 vs 6.60-6.91 vs 6.73-6.76 ms, profiles/r4/agg_grid_ab);
// set from Tunables.agg_insert_grid (MR_AGG_INSERT_GRID) by the binding
static unsigned g_ins_cap = 65536u;
// agg_combine_kernel<BATCH> (Tunables.agg_batch, MR_AGG_BATCH)
static bool g_agg_batch = false;
// agg_combine_kernel<false, PH> (Tunables.agg_phases, MR_AGG_PHASES)
static int g_agg_phases = 1;

extern "C" {

int mr_agg_set_insert_grid(int cap) {
  if (cap < 256) return -1;
  g_ins_cap = (unsigned)cap;
  return 0;
}

int mr_agg_set_batch(int on) {
  g_agg_batch = on != 0;
  return 0;
}

int mr_agg_set_phases(int ph) {
  if (ph != 1 && ph != 2 && ph != 4) return -1;
  g_agg_phases = ph;
  return 0;
}

// Keys pre-encoded (hi, lo, rep + rep_add) — or, when `text` is given, byte
// spans (starts int64, lens int32) of `text`, whose rep offsets are
// rep_base + start.  `src`: the byte source every rep word of the table
// indexes (long-key byte verification).
int mr_agg_insert(void* tag, void* thi, void* tlo, void* tval, void* trep, void* ctrl, u64 cap, const void* src,
                  const void* hi, const void* lo, const void* rep, u64 rep_add, const void* text, const void* starts,
                  const void* lens, u64 rep_base, u64 n, const void* cols, hipStream_t stream) {
  if (n == 0) return 0;
  const ColsArg* a = (const ColsArg*)cols;
  if (a->k < 0 || a->k > MAXC || (a->list && a->k < 1)) return -1;
  Keys ks;
  ks.hi = (const u64*)hi;
  ks.lo = (const u64*)lo;
  ks.rep = (const u64*)rep;
  ks.rep_add = rep_add;
  ks.text = (const u8*)text;
  ks.starts = (const long long*)starts;
  ks.lens = (const int*)lens;
  ks.rep_base = rep_base;
  if (!ks.text && (!ks.hi || !ks.lo)) return -2;
  if (!a->list && !a->rows_only && a->k > 0 && n >= (u64)CB_ROWS) {
    const size_t lds = (size_t)CB_SLOTS * (4 + (size_t)a->k) * sizeof(u64);
    static bool lds_attr = false;  // dynamic LDS above 64 KiB (k > 4 columns) must be allowed once
    if (!lds_attr) {
      for (const void* f : {(const void*)agg_combine_kernel<false, 1>, (const void*)agg_combine_kernel<false, 2>,
                            (const void*)agg_combine_kernel<false, 4>, (const void*)agg_combine_kernel<true, 1>})
        (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)((size_t)CB_SLOTS * (4 + MAXC) * sizeof(u64)));
      lds_attr = true;
    }
    // rows per block: 4096, or fewer (down to 512) so the grid has >= 1024 blocks
    u32 rows = (u32)CB_ROWS;
    while (rows > (u32)CB_T && (n + rows - 1) / rows < 1024) rows >>= 1;
    const u64 nb = (n + rows - 1) / rows;
    const GTab gt = ag_gtab(tag, thi, tlo, tval, trep, ctrl, cap, src);
    if (g_agg_batch)
      hipLaunchKernelGGL((agg_combine_kernel<true, 1>), dim3((unsigned)nb), dim3(CB_T), lds, stream, gt, ks, n,
                         to_cols(a), rows);
    else if (g_agg_phases == 2)
      hipLaunchKernelGGL((agg_combine_kernel<false, 2>), dim3((unsigned)nb), dim3(CB_T), lds, stream, gt, ks, n,
                         to_cols(a), rows);
    else if (g_agg_phases == 4)
      hipLaunchKernelGGL((agg_combine_kernel<false, 4>), dim3((unsigned)nb), dim3(CB_T), lds, stream, gt, ks, n,
                         to_cols(a), rows);
    else
      hipLaunchKernelGGL((agg_combine_kernel<false, 1>), dim3((unsigned)nb), dim3(CB_T), lds, stream, gt, ks, n,
                         to_cols(a), rows);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(agg_insert_kernel, dim3(ag_grid(n, 256, g_ins_cap)), dim3(256), 0, stream,
                     ag_gtab(tag, thi, tlo, tval, trep, ctrl, cap, src), ks, n, to_cols(a));
  return (int)hipGetLastError();
}

static int g_csv_tiles = 0, g_csv_mode = 0;

// Host-side mirror of CsvSpec.
struct CsvArg {
  long long sep, kf, nin;
  long long vf[MAXC];
  long long pin[MAXC];
};

// The fused CSV fold of text[0, n) into a fold-mode table (see csv_fold_kernel);
// rows_out (u64, device): += rows folded.
int mr_csv_fold(void* tag, void* thi, void* tlo, void* tval, void* trep, void* ctrl, u64 cap, const void* src,
                const void* text, u64 n, u64 rep_base, const void* spec, const void* cols, void* rows_out,
                hipStream_t stream) {
  if (n == 0) return 0;
  const ColsArg* a = (const ColsArg*)cols;
  const CsvArg* sa = (const CsvArg*)spec;
  if (a->list || a->k < 1 || a->k > MAXC || sa->nin < 0 || sa->nin > CV_MAXV) return -1;
  CsvSpec sp;
  sp.sep = (int)sa->sep;
  sp.kf = (int)sa->kf;
  sp.nin = (int)sa->nin;
  for (int j = 0; j < MAXC; ++j) {
    sp.vf[j] = (int)sa->vf[j];
    sp.pin[j] = (int)sa->pin[j];
    if (j < a->k && sp.pin[j] >= sp.nin) return -1;
  }
  const size_t lds = (size_t)CB_SLOTS * (4 + (size_t)a->k) * sizeof(u64);
  static bool lds_attr = false;
  if (!lds_attr) {
    (void)hipFuncSetAttribute((const void*)csv_fold_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)((size_t)CB_SLOTS * (4 + MAXC) * sizeof(u64)));
    lds_attr = true;
  }
  const u64 ntiles = (n + CV_TILE - 1) / CV_TILE;
  u32 tiles = 4;  // 32 KiB per block, fewer when that leaves the chip short of blocks
  while (tiles > 1 && (ntiles + tiles - 1) / tiles < 1024) tiles >>= 1;
  if (g_csv_tiles > 0) tiles = (u32)g_csv_tiles;
  const u64 nb = (ntiles + tiles - 1) / tiles;
  hipLaunchKernelGGL(csv_fold_kernel, dim3((unsigned)nb), dim3(CB_T), lds, stream,
                     ag_gtab(tag, thi, tlo, tval, trep, ctrl, cap, src), (const u8*)text, n, rep_base, sp, to_cols(a),
                     tiles, (unsigned long long*)rows_out, g_csv_mode);
  return (int)hipGetLastError();
}

// Launch knobs of mr_csv_fold: tiles per block (0 = auto) and an ablation
// mode (0 = normal, 1 = parse only, 2 = no LDS combine).
int mr_csv_set_config(int tiles, int mode) {
  if (tiles < 0 || tiles > 64 || mode < 0 || mode > 2) return -1;
  g_csv_tiles = tiles;
  g_csv_mode = mode;
  return 0;
}

// ghist: zeroed u32 [8][256] (the first 4 rows are filled); nshort: zeroed u64
int mr_slot_compact(void* tag, void* thi, void* tlo, void* tval, void* trep, void* ctrl, u64 cap, void* out_slot,
                    void* out_hi, void* out_lo, void* out_rep, void* counter, hipStream_t stream) {
  const u64 nb = (cap + 256 * SC_ITEMS - 1) / (256 * SC_ITEMS);
  hipLaunchKernelGGL(slot_compact_kernel, dim3((unsigned)nb), dim3(256), 0, stream,
                     ag_gtab(tag, thi, tlo, tval, trep, ctrl, cap, nullptr), cap, (long long*)out_slot,
                     (u64*)out_hi, (u64*)out_lo, (u64*)out_rep, (unsigned long long*)counter);
  return (int)hipGetLastError();
}

int mr_col_fill(void* col, u64 n, long long bits, int width, hipStream_t stream) {
  if (n == 0) return 0;
  if (width != 4 && width != 8) return -1;
  hipLaunchKernelGGL(col_fill_kernel, dim3(ag_grid(n, 256)), dim3(256), 0, stream, col, n, bits, width);
  return (int)hipGetLastError();
}

}  // extern "C"
