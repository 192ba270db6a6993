// invidx.hip — inverted-index build kernels (gfx950): word -> sorted list of
// the documents (lines) it occurs in.  The BASELINE "inverted-index build on
// the same corpus shape" workload: a MapReduce whose map emits a variable
// number of (word, doc) pairs per line and whose reduce concatenates them
// (reference hot loops K1-K4 and the segmented concat of K8, SURVEY.md §2.2;
// the emit/group machinery is job.lua:83-97 and utils.lua:206-271).
//
// Device formulation: every token becomes ONE 64-bit posting key
//     (dest << (slot_bits + doc_bits)) | (word_slot << doc_bits) | doc
// where word_slot is the word's slot in the HBM hash table (a dense key id),
// doc the line index and dest the owning rank (added after the map).  A radix
// sort of those keys groups by destination, then word, then document — exactly
// the shuffle + k-way merge of the reference — and one count + scatter pass
// (gw_*) drops adjacent duplicates (a word repeated in one line) and cuts the
// sorted postings into per-word lists.
//
// ii_map_kernel (one 512-thread workgroup per chunk, 8 KiB tiles):
//   1. stage the tile + halo into LDS with a whitespace bitmap and a newline
//      bitmap (16 bytes per thread);
//   2. per-thread newline prefix (wave scan + cross-wave LDS) -> every token's
//      line without any per-byte loop;
//   3. tokens probe a 4096-slot LDS table (exact 128-bit keys) — a chunk's
//      vocabulary costs one HBM insert per distinct word, not per token;
//      LDS misses (table 3/4 full) insert into HBM directly;
//   4. newly claimed LDS slots get their global slot (one gtab_insert each,
//      OP_NONE: the vocabulary folds no value, so a present word costs a load);
//   5. the tile's tokens are written at their text-order positions: a token's
//      output index = its chunk's token base (count_lines_tokens_kernel + an
//      exclusive scan, before the launch) + the tokens before it in the chunk
//      (block scans of per-thread token counts).  The posting array is thus in
//      line order, and a STABLE radix sort of the word bits alone (sort_keys
//      from_bit = doc_bits) yields (word, line) order: 3 passes for 21-bit word
//      ids instead of 6 over (word, line).
#include <hip/hip_runtime.h>
#include "mr_common.h"
#include "hashtab.h"

MR_LONG_MASK_SYMBOL(invidx)

namespace mr {
namespace ii {

constexpr int T = 512;
constexpr int SEG = 16;
constexpr int TILE = T * SEG;           // 8192 bytes
constexpr int PAD = 16;
constexpr int HALO = 64;
constexpr int STAGED = TILE + HALO;
constexpr int TXT = PAD + STAGED + 32;
constexpr int WSW = STAGED / 32 + 2;
// 2048 slots and 2048 buffered tokens keep the LDS at ~77 KiB: TWO workgroups
// per CU (one tile per workgroup by default: ~880 distinct words per tile)
constexpr int SLOTS = 2048;
constexpr int CLAIM_LIMIT = SLOTS * 3 / 4;
constexpr int PROBES = 32;
// a tile holds up to TILE/2 (+1) tokens; tokens past MAX_TOK (tiles of one-letter
// words) are resolved and written directly (one global atomic each)
constexpr int MAX_TOK = 2048;
constexpr u32 GFLAG = 0x80000000u;      // token ref is a global slot (LDS miss)
constexpr u32 UNRESOLVED = 0xFFFFFFFFu;

struct Lds {
  u8 txt[TXT];
  u32 ws[WSW];
  u32 tag[SLOTS];
  u32 rep[SLOTS];    // chunk-relative offset | len << 16 (len < 65536)
  u32 gslot[SLOTS];
  u64 hi[SLOTS];
  u64 lo[SLOTS];
  u32 tok_ref[MAX_TOK + 8];
  u16 tok_line[MAX_TOK + 8];  // line - the tile's first line (< TILE)
  u32 wave_nl[T / 64];
  u32 wave_tok[T / 64];
  u32 nclaimed;
};
static_assert(sizeof(Lds) <= 160 * 1024, "LDS budget");

__device__ __forceinline__ u32 mask16(uint4 q, u32 c0, bool ws) {
  u32 m = 0;
  const u32 w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const u32 b = (w[k] >> (8 * j)) & 0xFFu;
      m |= (ws ? (is_ws(b) ? 1u : 0u) : (b == c0 ? 1u : 0u)) << (4 * k + j);
    }
  return m;
}

__device__ __forceinline__ u32 funnel(u32 a, u32 b, u32 r8) { return r8 ? ((a >> r8) | (b << (32 - r8))) : a; }

__device__ u64 long_lo_global(const u8* text, u64 p0, u64 len) {
  u64 h = long_hash_init(len);
  for (u64 w = 0; w < len; w += 8) {
    const u64 n = (len - w) < 8 ? (len - w) : 8;
    const u64 word = load_word_le(text + p0 + w, n);
    h = long_hash_step(h, word);
  }
  return long_lo(h, mr_long_mask);
}

// LDS probe/claim; returns the local slot or -1 (table full / probe budget).
// A long key matched on (hi, lo) is compared byte for byte with the slot's
// first occurrence (both in this chunk, kb = its first byte): exact identity.
__device__ __forceinline__ int lds_find_or_claim(Lds& L, u64 hi, u64 lo, u32 rep, const u8* kb) {
  u64 h = hi ^ (lo * 0x9E3779B97F4A7C15ull);
  h ^= h >> 31;
  h *= 0xC2B2AE3D27D4EB4Full;
  h ^= h >> 29;
  const u32 tag = (u32)(h >> 32) | 1u;
  u32 slot = (u32)h & (SLOTS - 1);
  for (int probes = 0; probes < PROBES;) {
    u32 cur = __hip_atomic_load(&L.tag[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (cur == 0) {
      if (__hip_atomic_load(&L.nclaimed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= (u32)CLAIM_LIMIT)
        return -1;
      u32 expected = 0;
      if (__hip_atomic_compare_exchange_strong(&L.tag[slot], &expected, tag, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP)) {
        L.hi[slot] = hi;
        L.rep[slot] = rep;
        __hip_atomic_fetch_add(&L.nclaimed, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_store(&L.lo[slot], lo, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        return (int)slot;
      }
      cur = expected;
    }
    if (cur == tag) {
      const u64 l = __hip_atomic_load(&L.lo[slot], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (l == 0) continue;  // being published by its claimer
      if (l == lo && L.hi[slot] == hi &&
          (!key_is_long(lo) || rep_bytes_equal(kb, make_rep(L.rep[slot] & 0xFFFFu, L.rep[slot] >> 16),
                                               make_rep(rep & 0xFFFFu, rep >> 16))))
        return (int)slot;
    }
    slot = (slot + 1) & (SLOTS - 1);
    ++probes;
  }
  return -1;
}

// Newlines per chunk (for the chunk line bases) and, with out_tok, token
// starts per chunk (a non-whitespace byte whose predecessor is whitespace or
// the start of the text: exactly the tokens ii_map_kernel's chunk owns).  Each
// thread walks chunk/256 consecutive bytes, so the byte before a 16-byte
// segment is the previous segment's last (one extra load per thread).
__global__ void __launch_bounds__(256) count_newlines_kernel(const u8* __restrict__ text, u64 nbytes, u64 chunk,
                                                             u32* __restrict__ out, u32* __restrict__ out_tok) {
  const u64 b0 = (u64)blockIdx.x * chunk;
  const u64 b1 = min(b0 + chunk, nbytes);
  const u64 per = chunk / 256;
  const u64 p0 = b0 + threadIdx.x * per;
  const u64 p1 = min(p0 + per, b1);
  u32 c = 0, ct = 0;
  u32 prev = (p0 == 0 || p0 >= b1) ? 1u : (is_ws(text[p0 - 1]) ? 1u : 0u);
  for (u64 p = p0; p < p1; p += 16) {
    if (p + 16 <= p1 && ((uintptr_t)(text + p) & 15) == 0) {
      const uint4 q = *reinterpret_cast<const uint4*>(text + p);
      c += __builtin_popcount(mask16(q, 10u, false));
      const u32 m = mask16(q, 0, true);
      ct += __builtin_popcount(~m & ((m << 1) | prev) & 0xFFFFu);
      prev = (m >> 15) & 1u;
    } else {
      for (u64 k = p; k < min(p + 16, p1); ++k) {
        const u32 w = is_ws(text[k]) ? 1u : 0u;
        c += text[k] == '\n';
        ct += (!w && prev) ? 1u : 0u;
        prev = w;
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    c += __shfl_xor(c, o);
    ct += __shfl_xor(ct, o);
  }
  __shared__ u32 part[4], tpart[4];
  if ((threadIdx.x & 63) == 0) {
    part[threadIdx.x >> 6] = c;
    tpart[threadIdx.x >> 6] = ct;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    out[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
    if (out_tok) out_tok[blockIdx.x] = tpart[0] + tpart[1] + tpart[2] + tpart[3];
  }
}

__global__ void __launch_bounds__(T) ii_map_kernel(const u8* __restrict__ text, u64 nbytes, u64 chunk_bytes,
                                                   u64 rep_base, const u32* __restrict__ chunk_line_base,
                                                   const u32* __restrict__ chunk_tok_base,
                                                   const u32* __restrict__ chunk_tok_count, GTab g, u32 doc_bits,
                                                   u64* __restrict__ out,
                                                   const unsigned long long* __restrict__ out_counter, u64 out_cap,
                                                   u32* __restrict__ err) {
  __shared__ __attribute__((aligned(16))) Lds L;
  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  const u64 chunk_begin = (u64)blockIdx.x * chunk_bytes;
  if (chunk_begin >= nbytes) return;
  const u64 chunk_end = min(chunk_begin + chunk_bytes, nbytes);
  for (int s = t; s < SLOTS; s += T) {
    L.tag[s] = 0;
    L.lo[s] = 0;
    L.gslot[s] = UNRESOLVED;
  }
  if (t == 0) {
    L.nclaimed = 0;
    L.txt[PAD - 1] = chunk_begin > 0 ? text[chunk_begin - 1] : (u8)' ';
    L.ws[WSW - 2] = 0xFFFFFFFFu;
    L.ws[WSW - 1] = 0xFFFFFFFFu;
  }
  u32 line_base = chunk_line_base[blockIdx.x];
  // this launch's first output slot (advanced after the launch) + the tokens
  // of the chunks before this one
  u64 tok_next = (u64)*out_counter + chunk_tok_base[blockIdx.x];
  const u64 tok_end = tok_next + chunk_tok_count[blockIdx.x];
  u16* ws16 = reinterpret_cast<u16*>(L.ws);
  const u32* txt32 = reinterpret_cast<const u32*>(L.txt);
  const int aligned = ((uintptr_t)text & 15) == 0;
  u32 claims = 0;
  for (u64 tile_base = chunk_begin; tile_base < chunk_end; tile_base += TILE) {
    // ---- 1. stage + bitmaps
    u32 nlm;
    {
      const u64 gpos = tile_base + (u64)t * SEG;
      uint4 q;
      if (aligned && gpos + SEG <= nbytes) {
        q = *reinterpret_cast<const uint4*>(text + gpos);
      } else {
        u32 w[4];
        for (int k = 0; k < 4; ++k) {
          w[k] = 0;
          for (int j = 0; j < 4; ++j) {
            const u64 p = gpos + 4 * k + j;
            w[k] |= (p < nbytes ? (u32)text[p] : 32u) << (8 * j);
          }
        }
        q = make_uint4(w[0], w[1], w[2], w[3]);
      }
      *reinterpret_cast<uint4*>(L.txt + PAD + t * SEG) = q;
      ws16[t] = (u16)mask16(q, 0, true);
      nlm = mask16(q, 10u, false);
      // newlines past the chunk end belong to the next chunk
      if (gpos >= chunk_end) nlm = 0;
      else if (chunk_end - gpos < 16) nlm &= (1u << (chunk_end - gpos)) - 1u;
      if (t < HALO / SEG) {
        const u64 gh = tile_base + TILE + (u64)t * SEG;
        u32 w[4];
        for (int k = 0; k < 4; ++k) {
          w[k] = 0;
          for (int j = 0; j < 4; ++j) {
            const u64 p = gh + 4 * k + j;
            w[k] |= (p < nbytes ? (u32)text[p] : 32u) << (8 * j);
          }
        }
        const uint4 hq = make_uint4(w[0], w[1], w[2], w[3]);
        *reinterpret_cast<uint4*>(L.txt + PAD + TILE + t * SEG) = hq;
        ws16[T + t] = (u16)mask16(hq, 0, true);
      }
    }
    // ---- 2. newline prefix: inclusive wave scan, then cross-wave bases
    const u32 mine = __builtin_popcount(nlm);
    u32 incl = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const u32 v = __shfl_up(incl, o);
      if (lane >= o) incl += v;
    }
    if (lane == 63) L.wave_nl[wave] = incl;
    __syncthreads();
    u32 wbase = 0, tile_nl = 0;
#pragma unroll
    for (int w = 0; w < T / 64; ++w) {
      const u32 c = L.wave_nl[w];
      wbase += w < wave ? c : 0;
      tile_nl += c;
    }
    const u32 thread_line = line_base + wbase + incl - mine;
    // ---- 3. tokens of this thread's segment, at their text-order indices
    const u64 seg_base = tile_base + (u64)t * SEG;
    u32 starts = 0;
    if (seg_base < chunk_end) {
      const u32 m = ws16[t];
      const u32 prev_ws = t ? ((ws16[t - 1] >> 15) & 1u) : (is_ws(L.txt[PAD - 1]) ? 1u : 0u);
      starts = (~m) & ((m << 1) | prev_ws) & 0xFFFFu;
      const u64 lim_own = chunk_end - seg_base;
      if (lim_own < 16) starts &= (1u << lim_own) - 1u;
    }
    const u32 tmine = __builtin_popcount(starts);
    u32 tincl = tmine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const u32 v = __shfl_up(tincl, o);
      if (lane >= o) tincl += v;
    }
    if (lane == 63) L.wave_tok[wave] = tincl;
    __syncthreads();
    u32 twbase = 0, tile_tok = 0;
#pragma unroll
    for (int w = 0; w < T / 64; ++w) {
      const u32 c = L.wave_tok[w];
      twbase += w < wave ? c : 0;
      tile_tok += c;
    }
    u32 k = twbase + tincl - tmine;  // tile-relative index of this thread's first token
    {
      while (starts) {
        const int i = __builtin_ctz(starts);
        starts &= starts - 1;
        const u32 p = (u32)t * SEG + i;
        u32 q = p + 1;
        u32 wd = L.ws[q >> 5] >> (q & 31);
        u32 end;
        if (wd) {
          end = q + __builtin_ctz(wd);
        } else {
          u32 k = (q >> 5) + 1;
          while (L.ws[k] == 0) ++k;
          end = 32 * k + __builtin_ctz(L.ws[k]);
        }
        u64 len = end - p;
        const u64 gpos = tile_base + p;
        const u32 b = PAD + p;
        const u32 a = b >> 2;
        const u32 r8 = (b & 3u) * 8u;
        const u32 x0 = txt32[a], x1 = txt32[a + 1], x2 = txt32[a + 2], x3 = txt32[a + 3], x4 = txt32[a + 4];
        const u64 le_hi = (u64)funnel(x0, x1, r8) | ((u64)funnel(x1, x2, r8) << 32);
        const u64 le_lo = (u64)funnel(x2, x3, r8) | ((u64)funnel(x3, x4, r8) << 32);
        u64 hi = __builtin_bswap64(le_hi);
        u64 lo;
        if (end >= (u32)STAGED) {
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
        const u32 line = thread_line + __builtin_popcount(nlm & ((1u << i) - 1u));
        int ls = len < 65536 ? lds_find_or_claim(L, hi, lo, (u32)(gpos - chunk_begin) | ((u32)len << 16),
                                                       text + chunk_begin)
                         : -1;
        u32 ref;
        if (ls >= 0) {
          ref = (u32)ls;
        } else {
          u64 gs = 0;
          const int r = gtab_insert(g, hi, lo, 1, make_rep(rep_base + gpos, len), OP_NONE, &gs);
          claims += r == 2;
          if (r == 0) gs = 0;  // table overflow: flagged in ctrl[1], host re-runs bigger
          ref = GFLAG | (u32)gs;
        }
        if (k < (u32)MAX_TOK) {
          L.tok_ref[k] = ref;
          L.tok_line[k] = (u16)(line - line_base);
        } else {  // past the buffer (tiles of one-letter words): resolved and written here
          u64 gs = ref & ~GFLAG;
          if (!(ref & GFLAG)) {
            const int r = gtab_insert(g, hi, lo, 1, make_rep(rep_base + gpos, len), OP_NONE, &gs);
            claims += r == 2;
            if (r == 0) gs = 0;
          }
          const u64 o = tok_next + k;
          if (o < out_cap) out[o] = (gs << doc_bits) | (u64)line;
          else atomicOr(err, 1u);
        }
        ++k;
      }
    }
    __syncthreads();
    // ---- 4. resolve the global slots of new LDS keys
    for (int s = t; s < SLOTS; s += T) {
      if (L.tag[s] != 0 && L.gslot[s] == UNRESOLVED) {
        const u32 r = L.rep[s];
        u64 gs = 0;
        const int rc = gtab_insert(g, L.hi[s], L.lo[s], 1, make_rep(rep_base + chunk_begin + (r & 0xFFFFu), r >> 16),
                                   OP_NONE, &gs);
        claims += rc == 2;
        L.gslot[s] = rc ? (u32)gs : 0u;
      }
    }
    if (t == 0 && tok_next + tile_tok > out_cap) atomicOr(err, 1u);
    __syncthreads();
    // ---- 5. write the tile's posting keys (text order)
    {
      const u32 n = min(tile_tok, (u32)MAX_TOK);
      for (u32 j = t; j < n; j += T) {
        const u32 ref = L.tok_ref[j];
        const u32 gs = (ref & GFLAG) ? (ref & ~GFLAG) : L.gslot[ref];
        if (tok_next + j < out_cap) out[tok_next + j] = ((u64)gs << doc_bits) | (u64)(line_base + L.tok_line[j]);
      }
    }
    line_base += tile_nl;
    tok_next += tile_tok;
    __syncthreads();
    if (t == 0) L.txt[PAD - 1] = L.txt[PAD + TILE - 1];
    __syncthreads();
  }
  // the chunk's tokens must be exactly the ones the count kernel found (their
  // output slots were reserved from those counts): bit 1 of err otherwise
  if (t == 0 && tok_next != tok_end) atomicOr(err, 2u);
  gtab_count_claims(g, claims);
}

// key |= dest[slot(key)] << shift, slot(key) = (key >> doc_bits) & slot_mask
__global__ void ii_add_dest_kernel(u64* __restrict__ keys, u64 n, const u32* __restrict__ dest, u32 doc_bits,
                                   u64 slot_mask, u32 shift) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const u64 k = keys[i];
    keys[i] = k | ((u64)dest[(k >> doc_bits) & slot_mask] << shift);
  }
}

// Unique sorted keys -> keep flags (1 at i if i == 0 or key[i] != key[i-1]).
// Fused "sorted keys -> distinct keys" (replaces flags + 3-launch scan +
// compact, which wrote and re-read two n-word arrays): uq_count_kernel counts
// the run heads of each 4096-key tile, the tile counts are scanned, and
// uq_scatter_kernel recomputes the heads in registers and writes them at the
// tile's offset + a block scan.  Keys are read twice, nothing else is stored.
constexpr int UQ_T = 256, UQ_ITEMS = 16, UQ_TILE = UQ_T * UQ_ITEMS;

// Coalesced: round r, lane t reads key tile0 + r*UQ_T + t; its predecessor is
// the neighbouring lane's key (lane 0 of a wave loads it).
__global__ void __launch_bounds__(UQ_T) uq_count_kernel(const u64* __restrict__ keys, u64 n, u32* __restrict__ tc) {
  const int t = threadIdx.x, lane = t & 63;
  const u64 tile0 = (u64)blockIdx.x * UQ_TILE;
  u32 c = 0;
#pragma unroll 4
  for (int r = 0; r < UQ_ITEMS; ++r) {
    const u64 i = tile0 + (u64)r * UQ_T + t;
    const u64 k = i < n ? keys[i] : 0;
    u64 prev = __shfl_up(k, 1);
    if (lane == 0) prev = (i > 0 && i - 1 < n) ? keys[i - 1] : ~k;
    c += (i < n && (i == 0 || k != prev)) ? 1u : 0u;
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  __shared__ u32 w[UQ_T / 64];
  if (lane == 0) w[t >> 6] = c;
  __syncthreads();
  if (t == 0) tc[blockIdx.x] = w[0] + w[1] + w[2] + w[3];
}

// The tile goes through LDS: coalesced load, each thread takes 16 contiguous
// keys (run heads + block scan = their order), the kept keys are packed in LDS
// and streamed out with coalesced stores.
__global__ void __launch_bounds__(UQ_T) uq_scatter_kernel(const u64* __restrict__ keys, u64 n,
                                                          const u32* __restrict__ tile_off, u64* __restrict__ out) {
  __shared__ u64 sk[UQ_TILE + 1];  // sk[0] = the key before the tile
  __shared__ u32 w[UQ_T / 64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const u64 tile0 = (u64)blockIdx.x * UQ_TILE;
#pragma unroll 4
  for (int r = 0; r < UQ_ITEMS; ++r) {
    const u64 i = tile0 + (u64)r * UQ_T + t;
    sk[1 + r * UQ_T + t] = i < n ? keys[i] : 0;
  }
  if (t == 0) sk[0] = tile0 > 0 ? keys[tile0 - 1] : ~keys[0];
  __syncthreads();
  u64 k[UQ_ITEMS];
  u32 m = 0;
  {
    u64 prev = sk[t * UQ_ITEMS];
#pragma unroll
    for (int j = 0; j < UQ_ITEMS; ++j) {
      k[j] = sk[1 + t * UQ_ITEMS + j];
      const u64 i = tile0 + (u64)t * UQ_ITEMS + j;
      if (i < n && k[j] != prev) m |= 1u << j;
      prev = k[j];
    }
  }
  const u32 c = __builtin_popcount(m);
  u32 incl = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const u32 y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) w[wave] = incl;
  __syncthreads();  // also: every thread has read its keys from sk
  u32 base = 0, total = 0;
#pragma unroll
  for (int x = 0; x < UQ_T / 64; ++x) {
    base += x < wave ? w[x] : 0u;
    total += w[x];
  }
  u32 o = base + incl - c;
#pragma unroll
  for (int j = 0; j < UQ_ITEMS; ++j)
    if (m & (1u << j)) sk[o++] = k[j];
  __syncthreads();
  const u64 ob = tile_off[blockIdx.x];
  for (u32 x = t; x < total; x += UQ_T) out[ob + x] = sk[x];
}

// Sorted posting keys -> word lists in one count + one scatter pass (replaces
// unique scatter + split + a device-wide scan of per-posting head flags + the
// head write: four passes over n keys).  Per 4096-key tile: kept postings
// (all, or the distinct ones for concat_unique) and word heads (the word part
// key >> doc_bits differs from the previous key's; a head is always kept) are
// counted; after a scan of the two small tile-count arrays the scatter writes
// every kept posting's doc id at its rank and every word's (slot, start).
__device__ __forceinline__ void gw_flags(u64 k, u64 prev, bool first, int unique, u32 doc_bits, bool& keep,
                                         bool& head) {
  keep = first || !unique || k != prev;
  head = first || (k >> doc_bits) != (prev >> doc_bits);
}

__global__ void __launch_bounds__(UQ_T) gw_count_kernel(const u64* __restrict__ keys, u64 n, u32 doc_bits, int unique,
                                                        u32* __restrict__ tc /* [2][tiles] */, u64 tiles) {
  const int t = threadIdx.x, lane = t & 63;
  const u64 tile0 = (u64)blockIdx.x * UQ_TILE;
  u32 ck = 0, ch = 0;
#pragma unroll 4
  for (int r = 0; r < UQ_ITEMS; ++r) {
    const u64 i = tile0 + (u64)r * UQ_T + t;
    const u64 k = i < n ? keys[i] : 0;
    u64 prev = __shfl_up(k, 1);
    if (lane == 0) prev = (i > 0 && i - 1 < n) ? keys[i - 1] : ~k;
    if (i < n) {
      bool keep, head;
      gw_flags(k, prev, i == 0, unique, doc_bits, keep, head);
      ck += keep ? 1u : 0u;
      ch += head ? 1u : 0u;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    ck += __shfl_xor(ck, o);
    ch += __shfl_xor(ch, o);
  }
  __shared__ u32 w[2][UQ_T / 64];
  if (lane == 0) {
    w[0][t >> 6] = ck;
    w[1][t >> 6] = ch;
  }
  __syncthreads();
  if (t == 0) {
    tc[blockIdx.x] = w[0][0] + w[0][1] + w[0][2] + w[0][3];
    tc[tiles + blockIdx.x] = w[1][0] + w[1][1] + w[1][2] + w[1][3];
  }
}

__device__ __forceinline__ u32 block_excl_256(u32 c, u32* w /* [4] */, u32& total) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  u32 incl = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const u32 y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) w[wave] = incl;
  __syncthreads();
  u32 base = 0;
  total = 0;
#pragma unroll
  for (int x = 0; x < UQ_T / 64; ++x) {
    base += x < wave ? w[x] : 0u;
    total += w[x];
  }
  return base + incl - c;
}

__global__ void __launch_bounds__(UQ_T) gw_scatter_kernel(const u64* __restrict__ keys, u64 n, u32 doc_bits,
                                                          long long doc_base, u64 slot_mask, int unique,
                                                          const u32* __restrict__ off /* [2][tiles] */, u64 tiles,
                                                          int* __restrict__ doc, long long* __restrict__ word_slot,
                                                          long long* __restrict__ word_start) {
  __shared__ u64 sk[UQ_TILE + 1];  // sk[0] = the key before the tile
  __shared__ int sd[UQ_TILE];
  __shared__ u32 w[2][UQ_T / 64];
  const int t = threadIdx.x;
  const u64 tile0 = (u64)blockIdx.x * UQ_TILE;
#pragma unroll 4
  for (int r = 0; r < UQ_ITEMS; ++r) {
    const u64 i = tile0 + (u64)r * UQ_T + t;
    sk[1 + r * UQ_T + t] = i < n ? keys[i] : 0;
  }
  if (t == 0) sk[0] = tile0 > 0 ? keys[tile0 - 1] : ~keys[0];
  __syncthreads();
  u64 k[UQ_ITEMS];
  u32 mk = 0, mh = 0;
  {
    u64 prev = sk[t * UQ_ITEMS];
#pragma unroll
    for (int j = 0; j < UQ_ITEMS; ++j) {
      k[j] = sk[1 + t * UQ_ITEMS + j];
      const u64 i = tile0 + (u64)t * UQ_ITEMS + j;
      if (i < n) {
        bool keep, head;
        gw_flags(k[j], prev, i == 0, unique, doc_bits, keep, head);
        mk |= (keep ? 1u : 0u) << j;
        mh |= (head ? 1u : 0u) << j;
      }
      prev = k[j];
    }
  }
  u32 tk, th;
  u32 ok = block_excl_256(__builtin_popcount(mk), w[0], tk);
  u32 oh = block_excl_256(__builtin_popcount(mh), w[1], th);
  const u64 base_k = off[blockIdx.x], base_h = off[tiles + blockIdx.x];
  const u64 dm = (1ull << doc_bits) - 1;
#pragma unroll
  for (int j = 0; j < UQ_ITEMS; ++j) {
    if (mk & (1u << j)) {
      if (mh & (1u << j)) {
        word_slot[base_h + oh] = (long long)((k[j] >> doc_bits) & slot_mask);
        word_start[base_h + oh] = (long long)(base_k + ok);
        ++oh;
      }
      sd[ok++] = (int)((long long)(k[j] & dm) + doc_base);
    }
  }
  __syncthreads();
  for (u32 x = t; x < tk; x += UQ_T) doc[base_k + x] = sd[x];
}

}  // namespace ii
}  // namespace mr

using namespace mr;

static inline unsigned grid_n(u64 n, unsigned block, unsigned cap = 4096) {
  u64 g = (n + block - 1) / block;
  if (g > cap) g = cap;
  return (unsigned)(g ? g : 1);
}

extern "C" {

int mr_ii_chunk_bytes() { return 32 * 1024; }

// Newlines (and, with out_tok, token starts) per chunk of `chunk` bytes.
int mr_count_newlines(const void* text, u64 nbytes, u64 chunk, void* out, void* out_tok, hipStream_t s) {
  if (nbytes == 0) return 0;
  if (chunk % 4096) return -1;  // 256 threads x whole 16-byte segments
  const u64 nb = (nbytes + chunk - 1) / chunk;
  hipLaunchKernelGGL(ii::count_newlines_kernel, dim3((unsigned)nb), dim3(256), 0, s, (const u8*)text, nbytes, chunk,
                     (u32*)out, (u32*)out_tok);
  return (int)hipGetLastError();
}

// *counter += *add (one thread): a posting sink's fill after a map launch.
__global__ void ii_advance_kernel(unsigned long long* counter, const unsigned* add) { *counter += *add; }
int mr_ii_advance(void* counter, const void* add, hipStream_t s) {
  hipLaunchKernelGGL(ii_advance_kernel, dim3(1), dim3(1), 0, s, (unsigned long long*)counter, (const unsigned*)add);
  return (int)hipGetLastError();
}

// chunk_tok_base: exclusive scan of the per-chunk token counts
// (mr_count_newlines); postings land at *out_counter + their text-order index
// (the caller advances *out_counter by the launch's token total afterwards).
int mr_ii_map(const void* text, u64 nbytes, u64 chunk, u64 rep_base, const void* chunk_line_base,
              const void* chunk_tok_base, const void* chunk_tok_count, void* tag, void* hi, void* lo, void* val,
              void* rep, void* ctrl, u64 cap, u32 doc_bits, void* out, void* out_counter, u64 out_cap, void* err,
              hipStream_t s) {
  if (nbytes == 0) return 0;
  if (chunk % ii::TILE) return -1;
  (void)hi, (void)lo, (void)val;  // (slot records: their fields are at tag)
  // the vocabulary's rep words index the caller's byte source
  GTab g = gtab_make(tag, val, ctrl, cap, (const u8*)text - rep_base);
  const u64 nb = (nbytes + chunk - 1) / chunk;
  hipLaunchKernelGGL(ii::ii_map_kernel, dim3((unsigned)nb), dim3(ii::T), 0, s, (const u8*)text, nbytes, chunk,
                     rep_base, (const u32*)chunk_line_base, (const u32*)chunk_tok_base,
                     (const u32*)chunk_tok_count, g, doc_bits, (u64*)out,
                     (const unsigned long long*)out_counter, out_cap, (u32*)err);
  return (int)hipGetLastError();
}

int mr_ii_add_dest(void* keys, u64 n, const void* dest, u32 doc_bits, u64 slot_mask, u32 shift, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(ii::ii_add_dest_kernel, dim3(grid_n(n, 256)), dim3(256), 0, s, (u64*)keys, n, (const u32*)dest,
                     doc_bits, slot_mask, shift);
  return (int)hipGetLastError();
}

u64 mr_ii_unique_tiles(u64 n) { return (n + ii::UQ_TILE - 1) / ii::UQ_TILE; }

// pass 1: per-tile head counts into tc[mr_ii_unique_tiles(n)]
int mr_ii_unique_count(const void* keys, u64 n, void* tc, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(ii::uq_count_kernel, dim3((unsigned)mr_ii_unique_tiles(n)), dim3(ii::UQ_T), 0, s,
                     (const u64*)keys, n, (u32*)tc);
  return (int)hipGetLastError();
}

// pass 2 (after an exclusive scan of tc into tile_off): write the distinct keys
int mr_ii_unique_scatter(const void* keys, u64 n, const void* tile_off, void* out, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(ii::uq_scatter_kernel, dim3((unsigned)mr_ii_unique_tiles(n)), dim3(ii::UQ_T), 0, s,
                     (const u64*)keys, n, (const u32*)tile_off, (u64*)out);
  return (int)hipGetLastError();
}

// word grouping of sorted posting keys: pass 1 fills tc[2][mr_ii_unique_tiles(n)]
int mr_ii_group_count(const void* keys, u64 n, u32 doc_bits, int unique, void* tc, hipStream_t s) {
  if (n == 0) return 0;
  const u64 tiles = mr_ii_unique_tiles(n);
  hipLaunchKernelGGL(ii::gw_count_kernel, dim3((unsigned)tiles), dim3(ii::UQ_T), 0, s, (const u64*)keys, n, doc_bits,
                     unique, (u32*)tc, tiles);
  return (int)hipGetLastError();
}

// pass 2 (after an exclusive scan of tc into off): doc ids of the kept postings,
// (slot, start) of every word
int mr_ii_group_scatter(const void* keys, u64 n, u32 doc_bits, long long doc_base, u64 slot_mask, int unique,
                        const void* off, void* doc, void* word_slot, void* word_start, hipStream_t s) {
  if (n == 0) return 0;
  const u64 tiles = mr_ii_unique_tiles(n);
  hipLaunchKernelGGL(ii::gw_scatter_kernel, dim3((unsigned)tiles), dim3(ii::UQ_T), 0, s, (const u64*)keys, n,
                     doc_bits, doc_base, slot_mask, unique, (const u32*)off, tiles, (int*)doc, (long long*)word_slot,
                     (long long*)word_start);
  return (int)hipGetLastError();
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Insert n keys, returning each key's slot (the receive-side merge of words
// arriving from several ranks).
namespace mr {
namespace ii {
__global__ void ii_insert_slots_kernel(GTab g, const u64* __restrict__ hi, const u64* __restrict__ lo,
                                       const u64* __restrict__ rep, u64 n, long long* __restrict__ out_slot) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  u32 claims = 0;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    u64 s = 0;
    const int r = gtab_insert(g, hi[i], lo[i], 1, rep[i], OP_NONE, &s);
    claims += r == 2;
    out_slot[i] = r ? (long long)s : -1;
  }
  gtab_count_claims(g, claims);
}
}  // namespace ii
}  // namespace mr

// src: the byte source of the rep words (received key bytes; null = no
// long-key byte verification)
extern "C" int mr_ii_insert_slots(void* tag, void* thi, void* tlo, void* val, void* trep, void* ctrl, u64 cap,
                                  const void* hi, const void* lo, const void* rep, u64 n, void* out_slot,
                                  const void* src, hipStream_t s) {
  if (n == 0) return 0;
  GTab g = gtab_make(tag, val, ctrl, cap, (const u8*)src);
  hipLaunchKernelGGL(ii::ii_insert_slots_kernel, dim3(grid_n(n, 256)), dim3(256), 0, s, g, (const u64*)hi,
                     (const u64*)lo, (const u64*)rep, n, (long long*)out_slot);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Segmented gather of posting lists into a new word order: word i of the
// output is word perm[i] of the input (new_off: nw+1 output offsets).  Load
// balanced by OUTPUT position: a block owns a fixed chunk of postings, finds
// the word of its first posting with one binary search, then walks the words
// that overlap its chunk, all threads copying each overlap (coalesced).  A
// frequent word spans many blocks; a block spans many rare words.  (The first
// version binary-searched the word of every posting: 19 dependent loads per
// posting, 0.8 ms for 46 M postings.)
namespace mr {
namespace ii {
constexpr int SG_T = 256;
constexpr u64 SG_CHUNK = 4096;
__global__ void __launch_bounds__(SG_T) ii_seg_gather_kernel(const u32* __restrict__ perm,
                                                             const long long* __restrict__ old_start,
                                                             const long long* __restrict__ new_off, u64 nw, u64 n,
                                                             u64 nw_in, u64 n_src,
                                                             const int* __restrict__ src, int* __restrict__ dst) {
  // n: output postings; nw_in / n_src: words / postings of the input lists
  // (a reduce round gathers a subset of the words: nw < nw_in, n < n_src)
  __shared__ u64 s_w;
  const u64 c0 = (u64)blockIdx.x * SG_CHUNK;
  const u64 c1 = c0 + SG_CHUNK < n ? c0 + SG_CHUNK : n;
  if (threadIdx.x == 0) {
    u64 a = 0, b = nw;  // largest i with new_off[i] <= c0
    while (b - a > 1) {
      const u64 m = (a + b) >> 1;
      if ((u64)new_off[m] <= c0) a = m;
      else b = m;
    }
    s_w = a;
  }
  __syncthreads();
  for (u64 w = s_w; w < nw; ++w) {
    const u64 ws = (u64)new_off[w], we = (u64)new_off[w + 1];
    if (ws >= c1) break;
    const u64 a = ws > c0 ? ws : c0, b = we < c1 ? we : c1;
    const u64 s0 = (u64)old_start[clamp_row(perm[w], nw_in)] + (a - ws);
    for (u64 j = a + threadIdx.x; j < b; j += SG_T) dst[j] = src[clamp_row(s0 + (j - a), n_src)];
  }
}
}  // namespace ii
}  // namespace mr

extern "C" int mr_ii_seg_gather(const void* perm, const void* old_start, const void* new_off, u64 nw, u64 n,
                                u64 nw_in, u64 n_src, const void* src, void* dst, hipStream_t s) {
  if (n == 0 || nw == 0) return 0;
  const u64 blocks = (n + ii::SG_CHUNK - 1) / ii::SG_CHUNK;
  hipLaunchKernelGGL(ii::ii_seg_gather_kernel, dim3((unsigned)blocks), dim3(ii::SG_T), 0, s, (const u32*)perm,
                     (const long long*)old_start, (const long long*)new_off, nw, n, nw_in, n_src, (const int*)src,
                     (int*)dst);
  return (int)hipGetLastError();
}
