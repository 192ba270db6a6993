// keyops.hip — generic key kernels of the MapReduce data plane on gfx950.
//
// What this replaces in the reference (/root/reference):
//   K2 tokenizer         examples/WordCount/mapfn.lua:5-7  (line:gmatch("[^%s]+")):
//                        per-token (key, rep) emit for map functions that need
//                        every occurrence (no combining), and an exact count
//   K4 map-side group-by job.lua:83-97 (result[key][N+1] = value): the generic
//                        (key, value) insert into the HBM hash table (hashtab.h)
//   K8/K11               table compaction, key lengths + exact FNV-1 partition
//                        (examples/WordCount/partitionfn.lua), key-byte gather
// The fused word-count map (tokenize + LDS combine + flush) is wordcount3.hip.
//
// Geometry of the token walkers: 256 threads (4 wave64) per workgroup; each
// thread owns 16 bytes of a 4 KiB tile (one global_load_dwordx4 per lane,
// fully coalesced); a workgroup walks `chunk_bytes` of input tile by tile.
#include <hip/hip_runtime.h>
#include "mr_common.h"
#include "hashtab.h"

MR_LONG_MASK_SYMBOL(keyops)

namespace mr {

constexpr int WC_THREADS = 256;
constexpr int WC_SEG = 16;                      // bytes per thread per tile
constexpr int WC_TILE = WC_THREADS * WC_SEG;    // 4096 bytes
constexpr int WC_PAD = 16;                      // front pad; txt[PAD-1] = byte before tile
constexpr int WC_HALO = 64;                     // bytes of the next tile staged in LDS

struct TxtView {
  const u8* text;
  u64 nbytes;
};

__device__ __forceinline__ u32 load_byte(const TxtView& v, u64 p) {
  return p < v.nbytes ? (u32)v.text[p] : 32u;
}

// 56-bit hash part of a long key, read straight from global memory (rare path).
__device__ u64 long_key_lo_global(const TxtView& v, u64 p0, u64 len) {
  u64 h = long_hash_init(len);
  for (u64 w = 0; w < len; w += 8) {
    const u64 n = (len - w) < 8 ? (len - w) : 8;
    const u64 word = load_word_le(v.text + p0 + w, n);
    h = long_hash_step(h, word);
  }
  return long_lo(h, mr_long_mask);
}

// Stage tile [tile_base, tile_base + TILE + HALO) into LDS (bytes past nbytes
// read as whitespace).  txt[PAD-1] must already hold the byte before the tile.
__device__ __forceinline__ void stage_tile(const TxtView& v, u64 tile_base, u8* txt, bool aligned) {
  const int t = threadIdx.x;
  const u64 g = tile_base + (u64)t * WC_SEG;
  uint4 q;
  if (aligned && g + WC_SEG <= v.nbytes) {
    q = *reinterpret_cast<const uint4*>(v.text + g);
  } else {
    u32 w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      w[k] = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) w[k] |= load_byte(v, g + 4 * k + j) << (8 * j);
    }
    q = make_uint4(w[0], w[1], w[2], w[3]);
  }
  *reinterpret_cast<uint4*>(txt + WC_PAD + t * WC_SEG) = q;
  if (t < WC_HALO / WC_SEG) {
    const u64 gh = tile_base + WC_TILE + (u64)t * WC_SEG;
    u32 w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      w[k] = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) w[k] |= load_byte(v, gh + 4 * k + j) << (8 * j);
    }
    *reinterpret_cast<uint4*>(txt + WC_PAD + WC_TILE + t * WC_SEG) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// Walk the tokens that START in this thread's 16-byte segment of the staged
// tile and that start before `own_end` (global offset).  For each one,
// fn(hi, lo, gpos, len) is called with the exact 128-bit key.
template <typename Fn>
__device__ __forceinline__ void for_each_token(const TxtView& v, u64 tile_base, const u8* txt, u64 own_end, Fn&& fn) {
  const int t = threadIdx.x;
  const int li0 = WC_PAD + t * WC_SEG;
  const uint4 q = *reinterpret_cast<const uint4*>(txt + li0);
  const u32 words[4] = {q.x, q.y, q.z, q.w};
  u32 wsmask = 0;  // bit i => byte i is whitespace
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const u32 c = (words[i >> 2] >> (8 * (i & 3))) & 0xFFu;
    wsmask |= (is_ws(c) ? 1u : 0u) << i;
  }
  const u32 prev_ws = is_ws(txt[li0 - 1]) ? 1u : 0u;
  u32 starts = (~wsmask) & ((wsmask << 1) | prev_ws) & 0xFFFFu;
  const u64 seg_base = tile_base + (u64)t * WC_SEG;
  if (seg_base >= own_end) return;
  const u64 lim_own = own_end - seg_base;  // starts at index >= this are not ours
  if (lim_own < 16) starts &= (1u << lim_own) - 1u;
  constexpr int LIM = WC_PAD + WC_TILE + WC_HALO;
  while (starts) {
    const int i = __builtin_ctz(starts);
    starts &= starts - 1;
    int li = li0 + i;
    u64 hi = 0, lo = 0;
    u32 k = 0;
    u32 c = txt[li];
    while (true) {
      if (k < 8) hi |= (u64)c << (56 - 8 * k);
      else if (k < 15) lo |= (u64)c << (56 - 8 * (k - 8));
      ++k;
      ++li;
      if (li >= LIM) break;
      c = txt[li];
      if (is_ws(c)) break;
    }
    const u64 gpos = seg_base + i;
    u64 len = k;
    if (li >= LIM) {  // token runs past the staged halo: finish it from global memory
      u64 p = gpos + len;
      while (p < v.nbytes && !is_ws(v.text[p])) ++p;
      len = p - gpos;
    }
    if (len <= (u64)PACK_MAX) {
      lo |= len;
    } else {
      lo = long_key_lo_global(v, gpos, len);
    }
    fn(hi, lo, gpos, len);
  }
}

// Per-token emit (no combining): writes one (hi, lo, rep) triple per token,
// appended with one atomic per wave.  Used by map functions that need every
// occurrence (inverted index: key + document of each token).
__global__ void __launch_bounds__(WC_THREADS) tokenize_kernel(TxtView v, u64 chunk_bytes, u64 rep_base, u64* out_hi,
                                                              u64* out_lo, u64* out_rep, u64 cap,
                                                              unsigned long long* counter, int aligned) {
  __shared__ __attribute__((aligned(16))) u8 txt[WC_PAD + WC_TILE + WC_HALO];
  const int t = threadIdx.x;
  const u64 chunk_begin = (u64)blockIdx.x * chunk_bytes;
  if (chunk_begin >= v.nbytes) return;
  const u64 chunk_end = min(chunk_begin + chunk_bytes, v.nbytes);
  if (t == 0) txt[WC_PAD - 1] = chunk_begin > 0 ? v.text[chunk_begin - 1] : (u8)' ';
  __syncthreads();
  for (u64 tile_base = chunk_begin; tile_base < chunk_end; tile_base += WC_TILE) {
    stage_tile(v, tile_base, txt, aligned != 0);
    __syncthreads();
    for_each_token(v, tile_base, txt, chunk_end, [&](u64 hi, u64 lo, u64 gpos, u64 len) {
      const unsigned long long idx = atomicAdd(counter, 1ull);
      if (idx < cap) {
        out_hi[idx] = hi;
        out_lo[idx] = lo;
        out_rep[idx] = make_rep(rep_base + gpos, len);
      }
    });
    __syncthreads();
    if (t == 0) txt[WC_PAD - 1] = txt[WC_PAD + WC_TILE - 1];
    __syncthreads();
  }
}

// Count tokens only (for sizing tokenize outputs exactly).
__global__ void __launch_bounds__(WC_THREADS) count_tokens_kernel(TxtView v, u64 chunk_bytes,
                                                                  unsigned long long* counter, int aligned) {
  __shared__ __attribute__((aligned(16))) u8 txt[WC_PAD + WC_TILE + WC_HALO];
  __shared__ u32 block_count;
  const int t = threadIdx.x;
  const u64 chunk_begin = (u64)blockIdx.x * chunk_bytes;
  if (chunk_begin >= v.nbytes) return;
  const u64 chunk_end = min(chunk_begin + chunk_bytes, v.nbytes);
  if (t == 0) {
    block_count = 0;
    txt[WC_PAD - 1] = chunk_begin > 0 ? v.text[chunk_begin - 1] : (u8)' ';
  }
  __syncthreads();
  u32 mine = 0;
  for (u64 tile_base = chunk_begin; tile_base < chunk_end; tile_base += WC_TILE) {
    stage_tile(v, tile_base, txt, aligned != 0);
    __syncthreads();
    const int li0 = WC_PAD + t * WC_SEG;
    const u64 seg_base = tile_base + (u64)t * WC_SEG;
    if (seg_base < chunk_end) {
      u32 wsmask = 0;
#pragma unroll
      for (int i = 0; i < 16; ++i) wsmask |= (is_ws(txt[li0 + i]) ? 1u : 0u) << i;
      u32 starts = (~wsmask) & ((wsmask << 1) | (is_ws(txt[li0 - 1]) ? 1u : 0u)) & 0xFFFFu;
      const u64 lim_own = chunk_end - seg_base;
      if (lim_own < 16) starts &= (1u << lim_own) - 1u;
      mine += __builtin_popcount(starts);
    }
    __syncthreads();
    if (t == 0) txt[WC_PAD - 1] = txt[WC_PAD + WC_TILE - 1];
    __syncthreads();
  }
  atomicAdd(&block_count, mine);
  __syncthreads();
  if (t == 0) atomicAdd(counter, (unsigned long long)block_count);
}

// ---------------------------------------------------------------------------
// Generic (key, value) insert, e.g. received shuffle records or batch emits.
__global__ void hash_agg_kernel(const u64* hi, const u64* lo, const long long* val, const u64* rep, u64 n, GTab g,
                               int op, u64 rep_add) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  u32 claims = 0;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const u64 r = rep ? rep[i] + (rep_add << REP_LEN_BITS) : 0;
    claims += gtab_insert(g, hi[i], lo[i], val ? val[i] : 1ll, r, op) == 2;
  }
  gtab_count_claims(g, claims);
}

// Compact occupied slots into dense arrays.  Each 256-thread block owns a
// contiguous range of 4096 slots: per-thread counts -> LDS scan -> ONE atomic
// per block for the output base (a per-wave atomic on one counter serialised
// ~3e4 same-address atomics: 0.4 ms for a 2M-slot table).
constexpr int CP_ITEMS = 16;
// Occupied slots -> dense rows, in slot order.  The block's CP_ITEMS x 256
// slots are ranked k-major (slot b0 + k*256 + t), so for each k the lanes of a
// wave write CONSECUTIVE rows: one ballot + popcount per (k, wave), a 64-entry
// scan of the (k, wave) counts in LDS, one atomic per block for its base.
// (The first version gave each thread a run of its own and wrote it lane by
// lane: every store of a wave hit a different line.)  ``out_aos`` (optional):
// the rows also as 32-byte records {hi, lo, val, rep}, so a later gather by a
// permutation reads one sector per row instead of one per column.
__global__ void __launch_bounds__(256) table_compact_kernel(GTab g, u64 cap, u64* out_hi, u64* out_lo,
                                                            long long* out_val, u64* out_rep,
                                                            unsigned long long* counter, u64* out_aos) {
  constexpr int NW = 256 / 64;
  __shared__ u32 wc[CP_ITEMS * NW];
  __shared__ unsigned long long base;
  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  const unsigned long long below = (1ull << lane) - 1ull;
  const u64 b0 = (u64)blockIdx.x * 256 * CP_ITEMS;
  u32 occ = 0;
  u32 rank[CP_ITEMS];
#pragma unroll
  for (int k = 0; k < CP_ITEMS; ++k) {
    const u64 i = b0 + (u64)k * 256 + t;
    const bool o = i < cap && g.s[i].tag != 0;
    occ |= (o ? 1u : 0u) << k;
    const unsigned long long m = __ballot(o);
    rank[k] = (u32)__popcll(m & below);
    if (lane == 0) wc[k * NW + wave] = (u32)__popcll(m);
  }
  __syncthreads();
  if (t < 64) {
    // exclusive scan of the CP_ITEMS * NW (k-major) counts by one wave
    const u32 c = t < CP_ITEMS * NW ? wc[t] : 0u;
    u32 incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const u32 v = __shfl_up(incl, o);
      if (lane >= o) incl += v;
    }
    if (t < CP_ITEMS * NW) wc[t] = incl - c;
    if (t == 63) base = atomicAdd(counter, (unsigned long long)incl);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < CP_ITEMS; ++k) {
    if (occ & (1u << k)) {
      const u64 i = b0 + (u64)k * 256 + t;
      const u64 o = base + wc[k * NW + wave] + rank[k];
      const u64 h = g.s[i].hi, l = g.s[i].lo, r = g.s[i].rep;
      const long long v = g.val[i];
      out_hi[o] = h;
      out_lo[o] = l;
      out_val[o] = v;
      out_rep[o] = r;
      if (out_aos) {
        typedef u64 v2u __attribute__((ext_vector_type(2)));
        v2u* q = reinterpret_cast<v2u*>(out_aos + 4 * o);
        q[0] = v2u{h, l};
        q[1] = v2u{(u64)v, r};
      }
    }
  }
}

// Rows of 32-byte records {hi, lo, val, rep} gathered by an int32 permutation
// into four columns (two 16-byte loads per row from one 32-byte record), and
// (olen given) the key lengths of the gathered rows (from lo / rep: no key
// bytes read).
__global__ void __launch_bounds__(256) gather_aos4_kernel(const u32* __restrict__ perm, u64 n,
                                                          const u64* __restrict__ aos, u64* o0, u64* o1, u64* o2,
                                                          u64* o3, long long* olen) {
  typedef u64 v2u __attribute__((ext_vector_type(2)));
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    u64 j = perm[i];
    j = j < n ? j : n - 1;
    const v2u* q = reinterpret_cast<const v2u*>(aos + 4 * j);
    const v2u a = q[0], b = q[1];
    o0[i] = a.x;
    o1[i] = a.y;
    o2[i] = b.x;
    o3[i] = b.y;
    if (olen) olen[i] = (long long)(key_is_long(a.y) ? rep_len(b.y) : packed_len(a.y));
  }
}

// Key length and (optional) FNV-1 partition of each key.  Long-key bytes are
// read from `src` at rep offsets.
// out_w1 (optional, with out_part): key bytes 8..15 as a big-endian word,
// zero past the key's end (key_word_kernel's word 1), from the same pass over
// a long key's bytes.  out_k7 (optional, with out_w1; nparts <= 256): the
// two words of a 15-pass exact sort of 7-bit (ASCII) keys, k7[i] = partition
// << 56 | bytes 0..7 as 7-bit digits, k7[n + i] = bytes 8..15 likewise (the
// same order as (partition, hi, w1) when no byte has its top bit set);
// *k7_bad |= 1 when some key's first 16 bytes have a byte >= 0x80.
__device__ __forceinline__ u64 pack7(u64 w, u32& top) {
  u64 r = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const u64 b = (w >> (56 - 8 * j)) & 0xFFull;
    top |= (u32)b;
    r = (r << 7) | (b & 0x7Full);
  }
  return r;
}

// Alphabet-adaptive exact sort words (ops.exact_key_perm): the 16 7-bit key
// bytes of k7 (key_meta's words) re-coded through `code` (a byte's rank among
// the byte values present, zero padding -> 0) as `bits`-bit digits, most
// significant first, after the partition's `pbits` bits: word 0 = partition |
// codes of bytes 0..c0-1 (c0 = (64 - pbits) / bits, left-aligned), word 1 =
// the codes of the rest (right-aligned).  The same order as k7 — codes keep
// the byte order — in fewer radix passes: 5-bit codes with a 4-bit partition
// are 8 + 3 passes instead of 8 + 7.
__global__ void pack_alpha_kernel(const u64* __restrict__ k7, u64 n, const u8* __restrict__ code, u32 bits, u32 pbits,
                                  u64* __restrict__ out) {
  __shared__ u8 cd[128];
  if (threadIdx.x < 128) cd[threadIdx.x] = code[threadIdx.x];
  __syncthreads();
  const u32 c0 = min((64u - pbits) / bits, 16u);
  const u32 used = pbits + c0 * bits;
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const u64 a = k7[i], b = k7[n + i];
    u64 w0 = pbits ? (a >> 56) : 0ull, w1 = 0;
#pragma unroll
    for (u32 j = 0; j < 16; ++j) {
      const u32 ch = (u32)((j < 8 ? a : b) >> (49 - 7 * (j & 7))) & 0x7Fu;
      const u64 c = cd[ch];
      if (j < c0) w0 = (w0 << bits) | c;
      else w1 = (w1 << bits) | c;
    }
    out[i] = used < 64 ? w0 << (64 - used) : w0;
    out[n + i] = w1;
  }
}

// The 7-bit byte values of a key word's 8 bytes marked present in an LDS
// byte table (plain stores: every writer writes 1; a presence mask kept in
// registers cost ~0.2 ms of VALU per 23 M keys).
__device__ __forceinline__ void alpha_mark(u64 w, volatile u8* seen) {
#pragma unroll
  for (int j = 0; j < 8; ++j) seen[(u32)(w >> (8 * j)) & 0x7Fu] = 1;
}

// alpha (optional, with out_k7): the byte values present in the keys' first
// 16 bytes (zero padding included) as a 128-bit mask, for the
// alphabet-adaptive sort words (mr_pack_alpha)
__global__ void key_meta_kernel(const u64* hi, const u64* lo, const u64* rep, u64 n, const u8* src, u32 nparts,
                                u32* out_part, long long* out_len, u64* out_w1, u64* out_k7, u32* k7_bad,
                                u32* alpha) {
  __shared__ u8 seen[128];
  if (alpha && threadIdx.x < 128) seen[threadIdx.x] = 0;
  if (alpha) __syncthreads();
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const u64 h = hi[i], l = lo[i];
    const bool lng = key_is_long(l);
    const u64 len = lng ? rep_len(rep[i]) : packed_len(l);
    if (out_len) out_len[i] = (long long)len;
    if (!out_part) continue;  // lengths only: no key bytes read
    u32 f = FNV_OFFSET;
    u64 w1 = 0;
    if (!lng) {
      for (u32 k = 0; k < len; ++k) f = fnv1_step(f, packed_byte(h, l, k));
      w1 = l & ~0xFFull;
    } else {
      const u8* p = src + rep_off(rep[i]);
      for (u64 k0 = 0; k0 < len; k0 += 16) {  // 16 loads in flight per batch
        u32 b[16];
#pragma unroll
        for (u64 j = 0; j < 16; ++j) b[j] = k0 + j < len ? (u32)p[k0 + j] : 0u;
#pragma unroll
        for (u64 j = 0; j < 16; ++j) {
          const u64 k = k0 + j;
          if (k < len) {
            f = fnv1_step(f, b[j]);
            if (k - 8 < 8) w1 |= (u64)b[j] << (8 * (15 - k));
          }
        }
      }
    }
    out_part[i] = nparts ? f % nparts : f;
    if (out_w1) out_w1[i] = w1;
    if (out_k7) {
      u32 top = 0;
      const u64 a = pack7(h, top), b = pack7(w1, top);
      out_k7[i] = ((u64)(nparts ? f % nparts : f) << 56) | a;
      out_k7[n + i] = b;
      if (top & 0x80u) atomicOr(k7_bad, 1u);
      if (alpha) {
        alpha_mark(h, seen);
        alpha_mark(w1, seen);
      }
    }
  }
  if (alpha) {  // (uniform: every thread reaches this point)
    __syncthreads();
    // the block's table as a 128-bit mask (two waves, a ballot each); one
    // memory-side OR per word only for bits not yet seen (after the first
    // few blocks the mask is complete: no atomics)
    if (threadIdx.x < 128) {
      const unsigned long long m = __ballot(seen[threadIdx.x] != 0);
      const int lane = threadIdx.x & 63, q = (threadIdx.x >> 6) * 2 + (lane >> 5);
      if ((lane & 31) == 0) {
        const u32 v = (u32)(m >> (lane & 32));
        if (v & ~__hip_atomic_load(&alpha[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicOr(&alpha[q], v);
      }
    }
  }
}

// Materialise key bytes: dst[off[i] .. off[i]+len) = bytes of key i.
__global__ void gather_key_bytes_kernel(const u64* hi, const u64* lo, const u64* rep, const long long* off, u64 n,
                                        const u8* src, u8* dst, u64 dst_cap) {
  // writes stop at dst_cap: offsets built from rows of a flagged (given-up)
  // sort may overrun the capacity bound, and must never write past it
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const u64 h = hi[i], l = lo[i];
    const u64 o = (u64)off[i];
    if (o >= dst_cap) continue;
    u8* d = dst + o;
    const u64 room = dst_cap - o;
    if (!key_is_long(l)) {
      const u32 len = packed_len(l);
      for (u32 k = 0; k < len && k < room; ++k) d[k] = (u8)packed_byte(h, l, k);
    } else {
      const u64 len = rep_len(rep[i]) < room ? rep_len(rep[i]) : room;
      const u8* p = src + rep_off(rep[i]);
      // 16 loads in flight per batch: a byte loop waits out one memory round
      // trip per byte (n-gram keys of 16-40 bytes)
      for (u64 k0 = 0; k0 < len; k0 += 16) {
        u8 b[16];
#pragma unroll
        for (u64 j = 0; j < 16; ++j) b[j] = k0 + j < len ? p[k0 + j] : (u8)0;
#pragma unroll
        for (u64 j = 0; j < 16; ++j)
          if (k0 + j < len) d[k0 + j] = b[j];
      }
    }
  }
}

// Streaming map (input larger than the HBM arena ring): after a round, the
// long keys whose rep words point into that round's arena slot
// [lo_off, hi_off) of `buf` get their bytes copied to the persistent key heap
// at the front of `buf` (bump allocator `heap[0]`, capacity heap_cap) and
// their rep re-pointed there, so the slot can be refilled by a later round.
// heap[1] is set when the heap is full (the host raises).
__global__ void table_rehome_kernel(GSlot* __restrict__ slots, u64 cap, u8* __restrict__ buf, u64 lo_off, u64 hi_off,
                                    unsigned long long* __restrict__ heap, u64 heap_cap) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += stride) {
    if (slots[i].tag == 0 || !key_is_long(slots[i].lo)) continue;
    const u64 r = slots[i].rep;
    const u64 o = rep_off(r), n = rep_len(r);
    if (o < lo_off || o >= hi_off) continue;
    const unsigned long long d = atomicAdd(&heap[0], (unsigned long long)n);
    if (d + n > heap_cap) {
      atomicOr(&heap[1], 1ull);
      continue;
    }
    for (u64 k = 0; k < n; ++k) buf[d + k] = buf[o + k];
    slots[i].rep = make_rep(d, n);
  }
}

// Reset a table in one launch: every key record zeroed whole (two 16-byte
// stores: writing only {tag, lo}, half of each 32-byte record, ran 1.05 ms
// for 2^26 slots against 0.72 for whole records — partial lines), val =
// init, ctrl = 0.
__global__ void table_reset_kernel(GSlot* slots, long long* val, u32* ctrl, u64 cap, long long init) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += stride) {
    ulonglong2* p = reinterpret_cast<ulonglong2*>(&slots[i]);
    p[0] = make_ulonglong2(0ull, 0ull);
    p[1] = make_ulonglong2(0ull, 0ull);
    val[i] = init;
  }
  if (blockIdx.x == 0)
    for (u32 w = threadIdx.x; w < CTRL_WORDS; w += blockDim.x) ctrl[w] = 0;
}

}  // namespace mr

// ---------------------------------------------------------------------------
// C ABI (called from Python through ctypes with torch-owned buffers; no
// allocation or synchronisation inside, so every launch is graph-capturable).
using namespace mr;

static inline GTab make_gtab(void* tag, void* hi, void* lo, void* val, void* rep, void* ctrl, u64 cap,
                             const void* src = nullptr) {
  GTab g = gtab_make(tag, val, ctrl, cap, (const u8*)src);
  return g;
}

static inline int grid_for(u64 n, int block, int maxg = 8192) {
  u64 g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > (u64)maxg) g = maxg;
  return (int)g;
}

// Word k of every key: its bytes [8k, 8k+8) big-endian, zero past the end
// (word 0 = hi; packed keys keep bytes 8..14 in lo's top 7 bytes; long keys
// read their bytes from src).  The columns of an exact bytewise key sort
// (with the key length as the least significant column: a prefix sorts
// first), for key sets whose long keys share long prefixes.
__global__ void key_word_kernel(const u64* __restrict__ hi, const u64* __restrict__ lo, const u64* __restrict__ rep,
                                const u8* __restrict__ src, u64 n, u32 k, u64* __restrict__ out) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const u64 l = lo[i];
    u64 w = 0;
    if (k == 0 && hi != nullptr) {
      w = hi[i];
    } else if (!key_is_long(l)) {
      w = k == 1 ? (l & ~0xFFull) : 0ull;
    } else {
      const u64 r = rep[i];
      const u64 off = rep_off(r), len = rep_len(r);
#pragma unroll
      for (u32 j = 0; j < 8; ++j) {
        const u64 b = 8ull * k + j;
        w = (w << 8) | (b < len ? (u64)src[off + b] : 0ull);
      }
    }
    out[i] = w;
  }
}

// Exact key order after the (partition, bytes 0-15[, min(len, 16)]) sort of
// ops.exact_key_perm: only keys sharing their first 16 bytes can still be out
// of order (long keys; without the length column also a key and the same key
// with trailing NUL bytes).  exact_hash_kernel gives every row a 64-bit hash
// of its sort columns; on those hashes in sorted order, exact_fix_kernel finds each
// run of equal hashes (one thread per run start) and insertion-sorts the run
// by the full key: (partition, bytes 0-15, and for two long keys their bytes
// from 16 on and their lengths; else min(len, 16)) — the order the columns
// give, refined, so a run that only collides on the hash stays sorted too.
// Runs longer than EX_RUN set *bad (the caller refines in rounds instead).
constexpr int EX_RUN = 64;

__global__ void exact_hash_kernel(const int* __restrict__ part, const u64* __restrict__ hi, const u64* __restrict__ w1,
                                  const long long* __restrict__ klen, u64 n, u64* __restrict__ out) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const u64 lc = !klen ? 0ull : (klen[i] < 16 ? (u64)klen[i] : 16ull);  // no klen: the length is not a sort column
    out[i] = fmix64((u64)(unsigned)part[i] * 0x9E3779B97F4A7C15ull ^ fmix64(hi[i] ^ fmix64(w1[i] + lc)));
  }
}

// a < b in the exact key order (rows of one partition run)
__device__ bool exact_less(const int* part, const u64* hi, const u64* w1, const long long* klen, const u64* rep,
                           const u8* src, u32 a, u32 b) {
  if (part[a] != part[b]) return (unsigned)part[a] < (unsigned)part[b];
  if (hi[a] != hi[b]) return hi[a] < hi[b];
  if (w1[a] != w1[b]) return w1[a] < w1[b];
  const u64 la = (u64)klen[a], lb = (u64)klen[b];
  if (la < 16 || lb < 16) return la < lb;  // bytes 0-15 equal: the shorter key is a prefix
  const u64 oa = rep_off(rep[a]), ob = rep_off(rep[b]);
  const u64 m = la < lb ? la : lb;
  for (u64 i = 16; i < m; i += 16) {
    u32 x[16], y[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      x[j] = i + j < m ? src[oa + i + j] : 0u;
      y[j] = i + j < m ? src[ob + i + j] : 0u;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (x[j] != y[j]) return x[j] < y[j];
  }
  return la < lb;
}

__global__ void exact_fix_kernel(const u64* __restrict__ sh, u32* __restrict__ perm, u64 n,
                                 const int* __restrict__ part, const u64* __restrict__ hi, const u64* __restrict__ w1,
                                 const long long* __restrict__ klen, const u64* __restrict__ rep,
                                 const u8* __restrict__ src, u32* __restrict__ bad) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i + 1 < n; i += stride) {
    const u64 h = sh[i];
    if (sh[i + 1] != h || (i > 0 && sh[i - 1] == h)) continue;  // not a run start
    u64 e = i + 2;
    while (e < n && sh[e] == h && e - i <= (u64)EX_RUN) ++e;
    if (e - i > (u64)EX_RUN) {
      atomicOr(bad, 1u);
      continue;
    }
    u32 r[EX_RUN];
    const int m = (int)(e - i);
    for (int a = 0; a < m; ++a) r[a] = perm[i + a];
    for (int a = 1; a < m; ++a) {
      const u32 x = r[a];
      int b = a;
      while (b > 0 && exact_less(part, hi, w1, klen, rep, src, x, r[b - 1])) {
        r[b] = r[b - 1];
        --b;
      }
      r[b] = x;
    }
    for (int a = 0; a < m; ++a) perm[i + a] = r[a];
  }
}

extern "C" {

int mr_count_tokens(const void* text, u64 nbytes, u64 chunk_bytes, void* counter, hipStream_t stream) {
  if (nbytes == 0) return 0;
  if (chunk_bytes % WC_TILE) return -1;
  TxtView v{(const u8*)text, nbytes};
  const u64 nblocks = (nbytes + chunk_bytes - 1) / chunk_bytes;
  const int aligned = ((uintptr_t)text & 15) == 0;
  hipLaunchKernelGGL(count_tokens_kernel, dim3((unsigned)nblocks), dim3(WC_THREADS), 0, stream, v, chunk_bytes,
                     (unsigned long long*)counter, aligned);
  return (int)hipGetLastError();
}

int mr_tokenize(const void* text, u64 nbytes, u64 chunk_bytes, u64 rep_base, void* out_hi, void* out_lo, void* out_rep,
                u64 cap, void* counter, hipStream_t stream) {
  if (nbytes == 0) return 0;
  if (chunk_bytes % WC_TILE) return -1;
  TxtView v{(const u8*)text, nbytes};
  const u64 nblocks = (nbytes + chunk_bytes - 1) / chunk_bytes;
  const int aligned = ((uintptr_t)text & 15) == 0;
  hipLaunchKernelGGL(tokenize_kernel, dim3((unsigned)nblocks), dim3(WC_THREADS), 0, stream, v, chunk_bytes, rep_base,
                     (u64*)out_hi, (u64*)out_lo, (u64*)out_rep, cap, (unsigned long long*)counter, aligned);
  return (int)hipGetLastError();
}

// src (may be null): the byte source the table's rep words index (after
// rep_add), for the exact identity of long keys (hashtab.h)
int mr_hash_agg(const void* hi, const void* lo, const void* val, const void* rep, u64 n, u64 rep_add, int op, void* tag,
                void* thi, void* tlo, void* tval, void* trep, void* ctrl, u64 cap, const void* src,
                hipStream_t stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(hash_agg_kernel, dim3(grid_for(n, 256)), dim3(256), 0, stream, (const u64*)hi, (const u64*)lo,
                     (const long long*)val, (const u64*)rep, n, make_gtab(tag, thi, tlo, tval, trep, ctrl, cap, src),
                     op, rep_add);
  return (int)hipGetLastError();
}

int mr_table_compact(void* tag, void* hi, void* lo, void* val, void* rep, void* ctrl, u64 cap, void* out_hi,
                     void* out_lo, void* out_val, void* out_rep, void* counter, void* out_aos, hipStream_t stream) {
  const u64 nb = (cap + 256 * CP_ITEMS - 1) / (256 * CP_ITEMS);
  hipLaunchKernelGGL(table_compact_kernel, dim3((unsigned)nb), dim3(256), 0, stream,
                     make_gtab(tag, hi, lo, val, rep, ctrl, cap), cap, (u64*)out_hi, (u64*)out_lo,
                     (long long*)out_val, (u64*)out_rep, (unsigned long long*)counter, (u64*)out_aos);
  return (int)hipGetLastError();
}

// out[c][i] = aos[perm[i]].c for the four columns {hi, lo, val, rep}
int mr_gather_aos4(const void* perm, u64 n, const void* aos, void* o0, void* o1, void* o2, void* o3, void* olen,
                   hipStream_t stream) {
  if (n == 0) return 0;
  const u64 g = (n + 255) / 256;
  hipLaunchKernelGGL(gather_aos4_kernel, dim3((unsigned)(g < 16384 ? g : 16384)), dim3(256), 0, stream,
                     (const u32*)perm, n, (const u64*)aos, (u64*)o0, (u64*)o1, (u64*)o2, (u64*)o3, (long long*)olen);
  return (int)hipGetLastError();
}

// slots: the table's key records (hashtab.h GSlot)
int mr_table_rehome(void* slots, u64 cap, void* buf, u64 lo_off, u64 hi_off, void* heap, u64 heap_cap,
                    hipStream_t stream) {
  hipLaunchKernelGGL(table_rehome_kernel, dim3(grid_for(cap, 256)), dim3(256), 0, stream, (GSlot*)slots, cap,
                     (u8*)buf, lo_off, hi_off, (unsigned long long*)heap, heap_cap);
  return (int)hipGetLastError();
}

int mr_table_reset(void* slots, void* val, void* ctrl, u64 cap, long long init, hipStream_t stream) {
  hipLaunchKernelGGL(table_reset_kernel, dim3(grid_for(cap, 256)), dim3(256), 0, stream, (GSlot*)slots,
                     (long long*)val, (u32*)ctrl, cap, init);
  return (int)hipGetLastError();
}

int mr_key_word(const void* hi, const void* lo, const void* rep, const void* src, u64 n, u32 k, void* out,
                hipStream_t stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(key_word_kernel, dim3(grid_for(n, 256)), dim3(256), 0, stream, (const u64*)hi, (const u64*)lo,
                     (const u64*)rep, (const u8*)src, n, k, (u64*)out);
  return (int)hipGetLastError();
}

int mr_key_meta(const void* hi, const void* lo, const void* rep, u64 n, const void* src, u32 nparts, void* out_part,
                void* out_len, void* out_w1, void* out_k7, void* k7_bad, void* alpha, hipStream_t stream) {
  if (n == 0) return 0;
  if (out_k7 && (!out_w1 || !out_part || !k7_bad || nparts == 0 || nparts > 256)) return -1;
  if (alpha && !out_k7) return -1;
  // one key per thread (no grid cap): a thread's keys are latency chains of
  // random key-byte loads, and a capped grid ran ~11 of them in series
  hipLaunchKernelGGL(key_meta_kernel, dim3(grid_for(n, 256, 1 << 20)), dim3(256), 0, stream, (const u64*)hi,
                     (const u64*)lo,
                     (const u64*)rep, n, (const u8*)src, nparts, (u32*)out_part, (long long*)out_len,
                     (u64*)out_w1, (u64*)out_k7, (u32*)k7_bad, (u32*)alpha);
  return (int)hipGetLastError();
}

// code: u8 [128]; out: u64 [2 x n]; 1 <= bits <= 7, pbits <= 8, the rest's
// (16 - c0) * bits <= 64
int mr_pack_alpha(const void* k7, u64 n, const void* code, u32 bits, u32 pbits, void* out, hipStream_t stream) {
  if (n == 0) return 0;
  if (bits < 1 || bits > 7 || pbits > 8) return -1;
  hipLaunchKernelGGL(pack_alpha_kernel, dim3(grid_for(n, 256)), dim3(256), 0, stream, (const u64*)k7, n,
                     (const u8*)code, bits, pbits, (u64*)out);
  return (int)hipGetLastError();
}

int mr_gather_key_bytes(const void* hi, const void* lo, const void* rep, const void* off, u64 n, const void* src,
                        void* dst, u64 dst_cap, hipStream_t stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(gather_key_bytes_kernel, dim3(grid_for(n, 256, 1 << 20)), dim3(256), 0, stream, (const u64*)hi,
                     (const u64*)lo, (const u64*)rep, (const long long*)off, n, (const u8*)src, (u8*)dst, dst_cap);
  return (int)hipGetLastError();
}

int mr_exact_hash(const void* part, const void* hi, const void* w1, const void* klen, u64 n, void* out,
                  hipStream_t stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(exact_hash_kernel, dim3(grid_for(n, 256)), dim3(256), 0, stream, (const int*)part,
                     (const u64*)hi, (const u64*)w1, (const long long*)klen, n, (u64*)out);
  return (int)hipGetLastError();
}

int mr_exact_fix(const void* sh, void* perm, u64 n, const void* part, const void* hi, const void* w1,
                 const void* klen, const void* rep, const void* src, void* bad, hipStream_t stream) {
  if (n < 2) return 0;
  hipLaunchKernelGGL(exact_fix_kernel, dim3(grid_for(n, 256)), dim3(256), 0, stream, (const u64*)sh, (u32*)perm, n,
                     (const int*)part, (const u64*)hi, (const u64*)w1, (const long long*)klen, (const u64*)rep,
                     (const u8*)src, (u32*)bad);
  return (int)hipGetLastError();
}

}  // extern "C"
