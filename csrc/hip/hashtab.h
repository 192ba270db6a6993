// hashtab.h — HBM-resident open-addressing hash table for (128-bit key -> int64
// value, rep) aggregation.  This is the MI355X replacement for the reference's
// map-side `result[key][N+1] = value` grouping (/root/reference/mapreduce/job.lua:83-97)
// combined with the combiner (job.lua:92-96,198-202): values are folded with
// an associative op at insert time instead of being appended to Lua tables.
//
// Layout: slot i's KEY is one 32-byte record {tag, lo, hi, rep} (four slots
// per 128-byte line): a probe, its key compare and a long key's byte check
// touch one line (the structure-of-arrays table touched 4: tag, lo, hi, rep —
// the bigram's agg_combine waited on 82 % of its cycles).  The
// values stay in their own array: the folds are memory-side atomics, which
// serialise per line, and a hot word's line takes an add from every
// workgroup's flush — with the value inside the record, every probe of the
// four keys sharing that line queued behind those adds (the resident map ran
// 4.0 instead of 2.0 ms; profiles/r6/aos/).  Plus a control block {nclaimed,
// overflow, claim shards}.  The Python side sees the record fields as strided
// views of one int64 [cap, 4] tensor (ops/primitives.HashTable).
//
// Concurrency protocol (agent scope, placement independent — guide §6 G16):
//   claim:   CAS tag 0 -> gtab_tag(hi,lo)           (relaxed, agent); for keys of <= 7
//            bytes the tag IS the key (mr_common.h) and a tag match is final
//   publish: sc1 stores of hi, rep ; fold value ; s_waitcnt vmcnt(0) ; sc1 store lo
//   lookup:  tag match -> load lo and hi (relaxed); lo==0 => not yet published, retry;
//            lo match -> compare hi; on mismatch re-check after an acquire fence;
//            a long key (lo low byte 0xFF) must also match byte for byte
//            through the rep words (exact identity, mr_common.h) — keys that
//            collide on (prefix, hash) take separate slots.
//   lo is never 0 for a valid key (mr_common.h), so lo doubles as "published".
#pragma once
#include <hip/hip_runtime.h>
#include "mr_common.h"

namespace mr {

struct alignas(32) GSlot {
  u64 tag;
  u64 lo;
  u64 hi;
  u64 rep;
};

struct GTab {
  GSlot* s;        // cap key records
  long long* val;  // cap values
  u32* ctrl;      // [0] = claimed slots (host-side inserts), [1] = overflow flag,
                  // [CTRL_SHARD0 + CTRL_STRIDE * s] = claim-count shard s (s < CTRL_SHARDS)
  u64 mask;       // capacity - 1 (capacity is a power of two)
  const u8* src;  // byte source every rep word of this table indexes (long-key
                  // verification); null = identity on (prefix, 56-bit hash)
};

// The host passes a table as (key records, values, ctrl): the record base
// arrives in the historical "tag" argument of the entry points.
__host__ inline GTab gtab_make(void* slots, void* val, void* ctrl, u64 cap, const void* src) {
  GTab g;
  g.s = static_cast<GSlot*>(slots);
  g.val = static_cast<long long*>(val);
  g.ctrl = static_cast<u32*>(ctrl);
  g.mask = cap - 1;
  g.src = static_cast<const u8*>(src);
  return g;
}

// Exact identity of a long key already matched on (tag, hi, lo): compare its
// bytes with the slot's (rep published before lo; re-read after an acquire
// fence on a mismatch, as hi below).
__device__ __forceinline__ bool gtab_long_equal(const GTab& t, u64 slot, u64 rep);

constexpr u32 GTAB_MAX_PROBES = 1u << 14;
// Claim counts go to 64 shards, each on its own 128-byte line: same-address
// device atomics serialise at the memory side (~12 ns each,
// tools/probe/atomic_probe.hip), and one counter took an add from every wave
// of every map launch.  The host sums the shards (HashTable.stats()).
constexpr u32 CTRL_SHARD0 = 32;
constexpr u32 CTRL_STRIDE = 32;
constexpr u32 CTRL_SHARDS = 64;
constexpr u32 CTRL_WORDS = CTRL_SHARD0 + CTRL_STRIDE * CTRL_SHARDS;

__device__ __forceinline__ u64 ld_agent(const u64* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(u64* p, u64 v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void fold_value(long long* p, long long v, int op) {
  if (op == OP_NONE) return;
  if (op == OP_MIN) atomicMin(p, v);
  else if (op == OP_MAX) atomicMax(p, v);
  else atomicAdd((unsigned long long*)p, (unsigned long long)v);
}

// Insert (hi,lo) with value v.  Returns 2 when this call claimed a new slot,
// 1 when it folded into an existing key, 0 when the probe budget is exhausted
// (overflow flag set; the host re-runs with a larger table).  ``out_slot``
// (optional) receives the key's slot index — a dense-ish key id.  Callers count
// claims locally and publish them with gtab_count_claims (one atomic per wave:
// a same-address atomic per claim serialised ~3e5 adds in the map kernel).
__device__ __forceinline__ int gtab_insert(const GTab& t, u64 hi, u64 lo, long long v, u64 rep, int op,
                                           u64* out_slot = nullptr) {
  const u64 tag = gtab_tag(hi, lo);
  const bool exact = gtab_tag_exact(tag);
  u64 slot = gtab_home(tag, t.mask);
  u32 probes = 0;
  while (probes < GTAB_MAX_PROBES) {
    GSlot& sl = t.s[slot];
    u64 cur = ld_agent(&sl.tag);
    if (cur == 0) {
      u64 expected = 0;
      if (__hip_atomic_compare_exchange_strong(&sl.tag, &expected, tag, __ATOMIC_RELAXED,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        // publish (guide §6 G16 R1): write-through (sc1) stores of the payload,
        // drain them with vmcnt(0), then the sc1 store of `lo` that readers poll —
        // no buffer_wbl2 L2 write-back (a release fence per new key cost ~1 ms
        // over the 3e5 claims of the benchmark corpus).
        st_agent(&sl.hi, hi);
        st_agent(&sl.rep, rep);
        fold_value(&t.val[slot], v, op);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        st_agent(&sl.lo, lo);
        if (out_slot) *out_slot = slot;
        return 2;
      }
      cur = expected;
    }
    if (cur == tag && exact) {  // the tag is the key: fold without waiting for the payload
      fold_value(&t.val[slot], v, op);
      if (out_slot) *out_slot = slot;
      return 1;
    }
    if (cur == tag) {
      // lo and hi in one round trip (profiles/r4/probe_lohi/).  The hi load is
      // not ordered after the lo load, so it may return the slot's value from
      // before the claimer published (a previous key of this slot: reset does
      // not clear hi).  A stale hi that MISMATCHES is re-read after the acquire
      // fence below; a stale hi that happens to EQUAL ours is accepted without
      // one — which needs the claimer's key to share our 56-bit tag (a hash of
      // hi and lo) and our lo while differing in hi, i.e. a 56-bit collision of
      // two keys' (hi, lo) hashes, ~2^-56 per probe pair.  Keys of <= 7 bytes
      // (exact tags) never get here; long keys still compare bytes.
      const u64 l = ld_agent(&sl.lo);
      u64 h = ld_agent(&sl.hi);
      if (l == 0) continue;  // claimed but not yet published: re-read this slot
      if (l == lo) {
        if (h != hi) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          h = ld_agent(&sl.hi);
        }
        if (h == hi && (!key_is_long(lo) || t.src == nullptr || gtab_long_equal(t, slot, rep))) {
          fold_value(&t.val[slot], v, op);
          if (out_slot) *out_slot = slot;
          return 1;
        }
      }
    }
    slot = (slot + 1) & t.mask;
    ++probes;
    // a full table: once any insert has run out of probes and flagged the
    // overflow, the others stop within 64 probes instead of walking their
    // whole budget (the host regrows the table and re-runs the map either
    // way; a cold first map of 23 M distinct keys into the default 2^16
    // slots took ~300 ms per launch)
    if ((probes & 63u) == 0 && __hip_atomic_load(&t.ctrl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return 0;
  }
  __hip_atomic_fetch_or(&t.ctrl[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return 0;
}

// Up to N keys of one thread at once (bit k of `todo`): their home slots'
// records are loaded together, keys found there are done (their slot in
// `slot`), empty home slots are claimed with all CASes issued together, one
// vmcnt drain after the claims' payload stores, then their publishing `lo`
// stores (the claim protocol above, batched: one thread's keys pay about three
// memory round trips together instead of three each).  No value is folded
// (the caller folds its own columns at `slot`).  Returns the keys done; the
// others (a home slot holding another key, a lost CAS, a long key found, a
// claim not yet published) take gtab_insert.  `claimed`: the keys this call
// claimed.
// (Keys B .. B+N-1 of the caller's M-entry arrays: a batch of N = 4 keeps the
// probe state in ~40 VGPRs, so a 512-thread kernel keeps two blocks per CU.)
template <int N, int B, int M>
__device__ __forceinline__ u32 gtab_find_or_claim_home(const GTab& t, const u64 (&hi_)[M], const u64 (&lo_)[M],
                                                       const u64 (&rep_)[M], u32 todo, u64 (&slot)[M], u32& claimed) {
  static_assert(B + N <= M, "batch past the arrays");
  const u64* hi = hi_ + B;
  const u64* lo = lo_ + B;
  const u64* rep = rep_ + B;
  todo = (todo >> B) & ((1u << N) - 1u);
  u64 tg[N], gt[N], gl[N], gh[N], sl_[N];
#pragma unroll
  for (int k = 0; k < N; ++k) {
    tg[k] = gtab_tag(hi[k], lo[k]);
    sl_[k] = gtab_home(tg[k], t.mask);
  }
#pragma unroll
  for (int k = 0; k < N; ++k) {
    gt[k] = gl[k] = gh[k] = 0;
    if (todo & (1u << k)) {
      const GSlot& sl = t.s[sl_[k]];
      gt[k] = ld_agent(&sl.tag);
      if (!gtab_tag_exact(tg[k])) {
        gl[k] = ld_agent(&sl.lo);
        gh[k] = ld_agent(&sl.hi);
      }
    }
  }
  u32 done = 0, cas = 0;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    if (!(todo & (1u << k))) continue;
    if (gt[k] == tg[k] && (gtab_tag_exact(tg[k]) || (gl[k] == lo[k] && gh[k] == hi[k] && !key_is_long(lo[k]))))
      done |= 1u << k;
    else if (gt[k] == 0)
      cas |= 1u << k;
  }
  u32 won = 0;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    if (cas & (1u << k)) {
      u64 expected = 0;
      if (__hip_atomic_compare_exchange_strong(&t.s[sl_[k]].tag, &expected, tg[k], __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT))
        won |= 1u << k;
    }
  }
  if (won) {
#pragma unroll
    for (int k = 0; k < N; ++k) {
      if (won & (1u << k)) {
        st_agent(&t.s[sl_[k]].hi, hi[k]);
        st_agent(&t.s[sl_[k]].rep, rep[k]);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < N; ++k)
      if (won & (1u << k)) st_agent(&t.s[sl_[k]].lo, lo[k]);
  }
#pragma unroll
  for (int k = 0; k < N; ++k) slot[B + k] = sl_[k];
  claimed = won << B;
  return (done | won) << B;
}

__device__ __forceinline__ bool gtab_long_equal(const GTab& t, u64 slot, u64 rep) {
  u64 r = ld_agent(&t.s[slot].rep);
  if (rep_bytes_equal(t.src, r, rep)) return true;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  r = ld_agent(&t.s[slot].rep);
  return rep_bytes_equal(t.src, r, rep);
}

// Wave-reduce per-lane claim counts and add them to a claim-count shard (call
// with the whole wave active, e.g. at kernel end).
__device__ __forceinline__ void gtab_count_claims(const GTab& t, u32 claims) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) claims += __shfl_xor(claims, o);
  if ((threadIdx.x & 63) == 0 && claims) {
    const u32 shard = (blockIdx.x * 4u + (threadIdx.x >> 6)) & (CTRL_SHARDS - 1);
    __hip_atomic_fetch_add(&t.ctrl[CTRL_SHARD0 + CTRL_STRIDE * shard], claims, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace mr
