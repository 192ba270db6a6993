// wordcount3.hip — third-generation fused word-count map kernel (gfx950).
//
// Same contract as the reference's hot loops K1-K5
// (examples/WordCount/mapfn.lua:4-7, job.lua:83-97, job.lua:92-96): tokenize a
// byte stream on Lua-%s whitespace, build exact 128-bit keys, combine in an LDS
// hash table, fold each workgroup's distinct words into the HBM table.
//
// One launch shape: 512 threads, 2048 LDS slots, one 8 KiB tile per
// workgroup (two workgroups per CU, so one's flush to HBM overlaps the other's
// tokenizing), dense token lists.  The other shapes and the timing-only
// ablation modes measured in rounds 1-2 (profiles/r2/map_kernel/, the
// per-workgroup phase stamps of profiles/r1/map_v3/) are archived as
// profiles/r3/pruned/map_configs/wc_map3_configs.patch.
//
// The flush folds ~0.63 (workgroup, distinct word) entries per token, one
// device-scope atomic add each (memory-side atomics, profiles/r3/map_pmc/),
// but it is not the bound: dropping three quarters of the flush saved 12 %
// of the kernel (profiles/r5/map_probe/).  The tile work — staging, masks,
// token list, LDS hash inserts — is, latency-bound at 4 waves per SIMD.
#include <hip/hip_runtime.h>
#include "mr_common.h"
#include "hashtab.h"

MR_LONG_MASK_SYMBOL(wc3)

namespace mr {
namespace v3 {

constexpr int SEG = 16;
constexpr int PAD = 16;   // txt[PAD-1] = byte before the tile
constexpr int HALO = 64;  // staged bytes of the next tile
constexpr int PROBES = 32;

template <int T, int SLOTS>
struct Lds {
  static constexpr int TILE = T * SEG;
  static constexpr int STAGED = TILE + HALO;
  static constexpr int TXT = PAD + STAGED + 32;
  static constexpr int WSW = STAGED / 32 + 2;
  static constexpr int MAXTOK = T * 4;  // dense token list of a tile (~2.7 tokens per 16 B of text)
  u8 txt[TXT];
  u32 ws[WSW];
  u16 tokpos[MAXTOK];
  u32 wsum[T / 64];
  u32 tnext;  // (DYN) the next unclaimed entry of the tile's token list
  u64 tag[SLOTS];  // gtab_tag-style: a packed key of <= 7 bytes IS its tag
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
};

__device__ __forceinline__ u32 ws_mask_word(u32 w) {
  u32 m = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) m |= (is_ws((w >> (8 * j)) & 0xFFu) ? 1u : 0u) << j;
  return m;
}

__device__ __forceinline__ u32 ws_mask16(uint4 q) {
  return ws_mask_word(q.x) | (ws_mask_word(q.y) << 4) | (ws_mask_word(q.z) << 8) | (ws_mask_word(q.w) << 12);
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

// 16 bytes at gpos (bytes past nbytes read as spaces)
__device__ __forceinline__ uint4 load16(const u8* __restrict__ text, u64 gpos, u64 nbytes, int aligned) {
  if (aligned && gpos + SEG <= nbytes) {
    typedef u32 v4u __attribute__((ext_vector_type(4)));
    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(text + gpos));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
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
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// LDS combine.  Tags are 64-bit: for a packed key of <= 7 bytes (the frequent
// words) the tag is the key itself (hi | len, gtab_tag in mr_common.h), so a
// hit is ONE LDS read and a claim publishes the key in its CAS; other keys use
// a hashed tag plus the published (hi, lo) check (lo released last).
// A long key (>= 16 bytes) matched on (hi, lo) is compared byte for byte with
// the slot's first occurrence (both inside this chunk, `kb` = its first byte):
// colliding long keys take separate slots (exact identity, mr_common.h).
template <int T, int SLOTS>
__device__ __forceinline__ bool lds_insert(Lds<T, SLOTS>& L, u64 hi, u64 lo, u32 rep, const u8* kb) {
  u64 h = hi ^ (lo * 0x9E3779B97F4A7C15ull);
  h ^= h >> 31;
  h *= 0xC2B2AE3D27D4EB4Full;
  h ^= h >> 29;
  const bool exact = (lo - 1 < 7) && (hi & 0xFFull) == 0;
  const u64 tag = exact ? (hi | lo) : ((h & ~0xFFull) | 0x80ull);
  u32 slot = (u32)(h >> 40) & (SLOTS - 1);
  constexpr u32 LIMIT = SLOTS * 3 / 4;
  for (int probes = 0; probes < PROBES;) {
    u64 cur = __hip_atomic_load(&L.tag[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (cur == 0) {
      if (__hip_atomic_load(&L.nclaimed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= LIMIT) return false;
      u64 expected = 0;
      if (__hip_atomic_compare_exchange_strong(&L.tag[slot], &expected, tag, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP)) {
        L.hi[slot] = hi;
        L.rep[slot] = rep;
        __hip_atomic_fetch_add(&L.cnt[slot], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(&L.nclaimed, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (exact) L.lo[slot] = lo;  // read only by the flush, after a barrier
        else __hip_atomic_store(&L.lo[slot], lo, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        return true;
      }
      cur = expected;
    }
    if (cur == tag) {
      if (exact) {  // the tag is the key
        __hip_atomic_fetch_add(&L.cnt[slot], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return true;
      }
      const u64 l = __hip_atomic_load(&L.lo[slot], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (l == 0) continue;  // claimer has not published yet: re-read this slot
      if (l == lo && L.hi[slot] == hi &&
          (!key_is_long(lo) || rep_bytes_equal(kb, make_rep(L.rep[slot] & 0xFFFFu, L.rep[slot] >> 16),
                                               make_rep(rep & 0xFFFFu, rep >> 16)))) {
        __hip_atomic_fetch_add(&L.cnt[slot], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return true;
      }
    }
    slot = (slot + 1) & (SLOTS - 1);
    ++probes;
  }
  return false;
}

// T threads, SLOTS LDS slots, TPC tiles of T*16 bytes per workgroup chunk.
// The tile's token starts are first compacted into an LDS list (block prefix
// scan of per-thread start counts) and the tokens processed from that list,
// lane i taking tokens i, i+T, ... — every lane busy in every iteration,
// instead of each lane walking the 0..8 tokens that start in its own 16 bytes
// (the wave would run as long as its busiest lane).
// STAMPS (tools/map_stamps.py, a separate instantiation): every wave records
// where its time goes — waits at the tile's workgroup barriers, staging, the
// start masks + scan, the token list, the token loop, the flush — as 8 u64
// (wall_clock64 ticks) at stamps[(block * waves + wave) * 8].
// DYN: the waves take the tile's token list 64 entries at a time from an LDS
// counter instead of each thread walking the entries t, t + T, ...: a wave
// whose tokens were cheap takes more (round-6 stamps: the slowest wave's token
// loop ran 40 % over its workgroup's mean, and a quarter of the waves' time
// was spent waiting at the tile's barriers; profiles/r6/map_stamps/).
template <int T, int SLOTS, int TPC, bool STAMPS = false, bool DYN = false>
__global__ void __launch_bounds__(T) wc_map3_kernel(const u8* __restrict__ text, u64 nbytes, u64 rep_base, GTab g,
                                                    Ovf ovf, int aligned, u64* __restrict__ stamps = nullptr) {
  using L_t = Lds<T, SLOTS>;
  constexpr int TILE = L_t::TILE;
  constexpr int STAGED = L_t::STAGED;
  constexpr int WSW = L_t::WSW;
  constexpr u64 CHUNK = (u64)TILE * TPC;
  __shared__ __attribute__((aligned(16))) L_t L;
  const int t = threadIdx.x;
  const u64 chunk_begin = (u64)blockIdx.x * CHUNK;
  if (chunk_begin >= nbytes) return;
  const u64 chunk_end = min(chunk_begin + CHUNK, nbytes);
  [[maybe_unused]] u64 st_bar = 0, st_stage = 0, st_scan = 0, st_list = 0, st_loop = 0, st_flush = 0, st_p = 0;
  auto clk = [&]() -> u64 {
    if constexpr (STAMPS) return wall_clock64();
    return 0;
  };
  [[maybe_unused]] const u64 st_t0 = clk();
  auto bar = [&]() {  // a workgroup barrier (timed under STAMPS)
    const u64 a = clk();
    __syncthreads();
    if constexpr (STAMPS) st_bar += clk() - a;
  };
  for (int s = t; s < SLOTS; s += T) {
    L.tag[s] = 0;
    L.cnt[s] = 0;
    L.lo[s] = 0;
  }
  if (t == 0) {
    L.nclaimed = 0;
    L.txt[PAD - 1] = chunk_begin > 0 ? text[chunk_begin - 1] : (u8)' ';
    L.ws[WSW - 2] = 0xFFFFFFFFu;
    L.ws[WSW - 1] = 0xFFFFFFFFu;
  }
  u32 claims = 0;
  u16* ws16 = reinterpret_cast<u16*>(L.ws);
  const u32* txt32 = reinterpret_cast<const u32*>(L.txt);
  constexpr int NH = HALO / SEG;
  // registers hold the NEXT tile's bytes while the current tile is processed
  uint4 q = load16(text, chunk_begin + (u64)t * SEG, nbytes, aligned);
  uint4 qh = make_uint4(0, 0, 0, 0);
  if (t < NH) qh = load16(text, chunk_begin + TILE + (u64)t * SEG, nbytes, aligned);
  for (u64 tile_base = chunk_begin; tile_base < chunk_end; tile_base += TILE) {
    // the byte before this tile: the last byte of the previous tile, which
    // thread T-1 held (nobody reads txt[PAD-1] between the previous tile's
    // final barrier and this tile's staging barrier)
    if (t == T - 1 && tile_base != chunk_begin) L.txt[PAD - 1] = L.txt[PAD + TILE - 1];
    bar();
    st_p = clk();
    *reinterpret_cast<uint4*>(L.txt + PAD + t * SEG) = q;
    ws16[t] = (u16)ws_mask16(q);
    if (t < NH) {
      *reinterpret_cast<uint4*>(L.txt + PAD + TILE + t * SEG) = qh;
      ws16[T + t] = (u16)ws_mask16(qh);
    }
    if constexpr (STAMPS) st_stage += clk() - st_p;
    bar();
    st_p = clk();
    const u64 next = tile_base + TILE;
    if (next < chunk_end) {  // prefetch: consumed after this tile's token loop
      q = load16(text, next + (u64)t * SEG, nbytes, aligned);
      if (t < NH) qh = load16(text, next + TILE + (u64)t * SEG, nbytes, aligned);
    }
    // one token starting at tile offset p
    auto process = [&](u32 p) {
      u32 qq = p + 1;
      u32 wd = L.ws[qq >> 5] >> (qq & 31);
      u32 end;
      if (wd) {
        end = qq + __builtin_ctz(wd);
      } else {
        u32 k = (qq >> 5) + 1;
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
      const bool ok = len < 65536 && lds_insert(L, hi, lo, (u32)(gpos - chunk_begin) | ((u32)len << 16),
                                                 text + chunk_begin);
      if (!ok) {
        const u64 grep = make_rep(rep_base + gpos, len);
        const unsigned long long idx = atomicAdd(ovf.counter, 1ull);
        if (idx < ovf.cap) {
          ovf.hi[idx] = hi;
          ovf.lo[idx] = lo;
          ovf.rep[idx] = grep;
        } else {
          claims += gtab_insert(g, hi, lo, 1, grep, OP_SUM) == 2;
        }
      }
    };
    const u64 seg_base = tile_base + (u64)t * SEG;
    u32 starts = 0;
    if (seg_base < chunk_end) {
      const u32 m = ws16[t];
      const u32 prev_ws = t ? ((ws16[t - 1] >> 15) & 1u) : (is_ws(L.txt[PAD - 1]) ? 1u : 0u);
      starts = (~m) & ((m << 1) | prev_ws) & 0xFFFFu;
      const u64 lim_own = chunk_end - seg_base;
      if (lim_own < 16) starts &= (1u << lim_own) - 1u;
    }
    {
      // block exclusive scan of the per-thread token counts
      constexpr int MAXTOK = L_t::MAXTOK;
      const int lane = t & 63, wave = t >> 6;
      const u32 c = __builtin_popcount(starts);
      u32 incl = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const u32 v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
      }
      if (lane == 63) L.wsum[wave] = incl;
      if (DYN && t == 0) L.tnext = 0;
      if constexpr (STAMPS) st_scan += clk() - st_p;
      bar();
      st_p = clk();
      u32 base = 0, total = 0;
#pragma unroll
      for (int w = 0; w < T / 64; ++w) {
        const u32 x = L.wsum[w];
        base += w < wave ? x : 0u;
        total += x;
      }
      u32 k = base + incl - c;
      while (starts) {
        const int i = __builtin_ctz(starts);
        starts &= starts - 1;
        if (k < (u32)MAXTOK) L.tokpos[k] = (u16)(t * SEG + i);
        else process((u32)t * SEG + i);  // a tile denser than the list (one-letter words): in place
        ++k;
      }
      if constexpr (STAMPS) st_list += clk() - st_p;
      bar();
      st_p = clk();
      const u32 ntok = total < (u32)MAXTOK ? total : (u32)MAXTOK;
      if constexpr (DYN) {
        for (;;) {
          u32 b0 = 0;
          if (lane == 0) b0 = __hip_atomic_fetch_add(&L.tnext, 64u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          b0 = __shfl(b0, 0);
          if (b0 >= ntok) break;
          if (b0 + lane < ntok) process(L.tokpos[b0 + lane]);
        }
      } else {
        for (u32 x = t; x < ntok; x += T) process(L.tokpos[x]);
      }
    }
    if constexpr (STAMPS) st_loop += clk() - st_p;
    bar();
  }
  [[maybe_unused]] const u64 st_f0 = clk();
  // flush: each thread folds its PER slots.  The common case is a key already
  // in the HBM table at its home slot, so tag/lo/hi of every home slot are
  // loaded speculatively in ONE batch (one memory round trip instead of a
  // dependent tag -> lo -> hi chain per key); a full match needs only the
  // atomic add, anything else takes the general gtab_insert path.
  constexpr int PER = SLOTS / T;
  static_assert(SLOTS % T == 0, "slots must be a multiple of the block size");
  u64 khi[PER], klo[PER], ktag[PER], kslot[PER], gt[PER], gl[PER], gh[PER];
  u32 kcnt[PER], krep[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int s = t + k * T;
    kcnt[k] = L.tag[s] != 0 ? L.cnt[s] : 0u;
    khi[k] = L.hi[s];
    klo[k] = L.lo[s];
    krep[k] = L.rep[s];
    ktag[k] = gtab_tag(khi[k], klo[k]);
    kslot[k] = gtab_home(ktag[k], g.mask);
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    if (kcnt[k]) {
      // (one slot record: tag, lo and hi share a line)
      gt[k] = ld_agent(&g.s[kslot[k]].tag);
      if (!gtab_tag_exact(ktag[k])) {
        gl[k] = ld_agent(&g.s[kslot[k]].lo);
        gh[k] = ld_agent(&g.s[kslot[k]].hi);
      } else {
        gl[k] = klo[k];
        gh[k] = khi[k];
      }
    }
  }
  // new keys whose home slot is empty are claimed in a batch too: all CASes,
  // one wait, all payload stores, ONE vmcnt drain, all publishing stores
  // (hashtab.h protocol) — a per-key claim costs two serial memory round
  // trips, and a cold table (first map of an iteration) is claim-heavy
  u32 state = 0;  // bit k: entry k is done
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    if (!kcnt[k]) {
      state |= 1u << k;
    } else if (gt[k] == ktag[k] && gl[k] == klo[k] && gh[k] == khi[k] && !key_is_long(klo[k])) {
      // (a long key takes gtab_insert below: its bytes are verified there)
      fold_value(&g.val[kslot[k]], (long long)kcnt[k], OP_SUM);
      state |= 1u << k;
    }
  }
  u32 won = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    if (!(state & (1u << k)) && gt[k] == 0) {
      u64 expected = 0;
      if (__hip_atomic_compare_exchange_strong(&g.s[kslot[k]].tag, &expected, ktag[k], __ATOMIC_RELAXED,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        won |= 1u << k;
    }
  }
  if (won) {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      if (won & (1u << k)) {
        const u32 r = krep[k];
        st_agent(&g.s[kslot[k]].hi, khi[k]);
        st_agent(&g.s[kslot[k]].rep, make_rep(rep_base + chunk_begin + (r & 0xFFFFu), r >> 16));
        fold_value(&g.val[kslot[k]], (long long)kcnt[k], OP_SUM);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < PER; ++k)
      if (won & (1u << k)) st_agent(&g.s[kslot[k]].lo, klo[k]);
    claims += __builtin_popcount(won);
    state |= won;
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    if (state & (1u << k)) continue;
    const u32 r = krep[k];
    claims += gtab_insert(g, khi[k], klo[k], (long long)kcnt[k],
                          make_rep(rep_base + chunk_begin + (r & 0xFFFFu), r >> 16), OP_SUM) == 2;
  }
  gtab_count_claims(g, claims);
  if constexpr (STAMPS) {
    const u64 now = clk();
    st_flush = now - st_f0;
    if ((t & 63) == 0) {
      u64* o = stamps + ((u64)blockIdx.x * (T / 64) + (t >> 6)) * 8;
      o[0] = now - st_t0;
      o[1] = st_bar;
      o[2] = st_stage;
      o[3] = st_scan;
      o[4] = st_list;
      o[5] = st_loop;
      o[6] = st_flush;
      o[7] = claims;
    }
  }
}

__global__ void __launch_bounds__(256) ovf_agg3_kernel(Ovf o, GTab g) {
  const unsigned long long n0 = *o.counter;
  const u64 n = n0 < o.cap ? n0 : o.cap;
  const u64 stride = (u64)gridDim.x * blockDim.x;
  u32 claims = 0;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    claims += gtab_insert(g, o.hi[i], o.lo[i], 1ll, o.rep[i], OP_SUM) == 2;
  gtab_count_claims(g, claims);
}

// (1024 slots, 45.5 KiB, would leave LDS on every CU for the W > 1 post-map
// kernels beside the map, but overflowed the table: resident map 4.25 vs
// 2.29 ms per step, W = 8 proxy 0.96 vs 0.71 ms; profiles/r5/proxy/slots/)
constexpr int MAP_T = 512, MAP_SLOTS = 2048, MAP_TPC = 1;
static_assert(sizeof(Lds<MAP_T, MAP_SLOTS>) <= 80 * 1024, "two workgroups per CU");
// (Wider combine spans — 4096 LDS slots over 32/64 KiB, one workgroup per CU —
// cut the flush's atomics by 18 % but ran 3.40 vs 2.04 ms; removed in round 5,
// archived in profiles/r5/pruned/, numbers in profiles/r4/map_shapes/.)

static int g_map_dyn = 1;  // mr_wc3_set_dyn (MR_MAP_DYN, default on): DYN token lists

template <int T, int SLOTS, int TPC>
static void launch_map3(const u8* text, u64 nbytes, u64 rep_base, const GTab& g, const Ovf& o, int aligned,
                        hipStream_t stream, u64* stamps = nullptr) {
  constexpr u64 CHUNK = (u64)T * SEG * TPC;
  const u64 nblocks = (nbytes + CHUNK - 1) / CHUNK;
  const dim3 grid((unsigned)nblocks), block(T);
  if (stamps && g_map_dyn)
    hipLaunchKernelGGL((wc_map3_kernel<T, SLOTS, TPC, true, true>), grid, block, 0, stream, text, nbytes, rep_base, g,
                       o, aligned, stamps);
  else if (stamps)
    hipLaunchKernelGGL((wc_map3_kernel<T, SLOTS, TPC, true>), grid, block, 0, stream, text, nbytes, rep_base, g, o,
                       aligned, stamps);
  else if (g_map_dyn)
    hipLaunchKernelGGL((wc_map3_kernel<T, SLOTS, TPC, false, true>), grid, block, 0, stream, text, nbytes, rep_base,
                       g, o, aligned, nullptr);
  else
    hipLaunchKernelGGL((wc_map3_kernel<T, SLOTS, TPC>), grid, block, 0, stream, text, nbytes, rep_base, g, o, aligned,
                       nullptr);
}

}  // namespace v3
}  // namespace mr

using namespace mr;

extern "C" {

int mr_wc3_set_dyn(int on) {
  v3::g_map_dyn = on ? 1 : 0;
  return 0;
}

int mr_wc_map3(const void* text, u64 nbytes, u64 rep_base, void* tag, void* hi, void* lo, void* val, void* rep,
               void* ctrl, u64 cap, void* ovf_hi, void* ovf_lo, void* ovf_rep, u64 ovf_cap, void* ovf_counter,
               hipStream_t stream) {
  if (nbytes == 0) return 0;
  (void)hi, (void)lo, (void)val;  // (slot records: their fields are at tag)
  // every rep word of this table indexes the caller's byte source
  GTab g = gtab_make(tag, val, ctrl, cap, (const u8*)text - rep_base);
  v3::Ovf o{(u64*)ovf_hi, (u64*)ovf_lo, (u64*)ovf_rep, ovf_cap, (unsigned long long*)ovf_counter};
  const int aligned = ((uintptr_t)text & 15) == 0;
  const u8* t = (const u8*)text;
  v3::launch_map3<v3::MAP_T, v3::MAP_SLOTS, v3::MAP_TPC>(t, nbytes, rep_base, g, o, aligned, stream);
  hipLaunchKernelGGL(v3::ovf_agg3_kernel, dim3(1024), dim3(256), 0, stream, o, g);
  return (int)hipGetLastError();
}

// The same map with per-wave phase stamps (diagnosis; tools/map_stamps.py):
// stamps = u64 [blocks * MAP_T / 64 * 8], blocks = ceil(nbytes / 8 KiB).
int mr_wc_map3_stamped(const void* text, u64 nbytes, u64 rep_base, void* tag, void* val, void* ctrl, u64 cap,
                       void* ovf_hi, void* ovf_lo, void* ovf_rep, u64 ovf_cap, void* ovf_counter, void* stamps,
                       hipStream_t stream) {
  if (nbytes == 0 || stamps == nullptr) return nbytes ? -1 : 0;
  GTab g = gtab_make(tag, val, ctrl, cap, (const u8*)text - rep_base);
  v3::Ovf o{(u64*)ovf_hi, (u64*)ovf_lo, (u64*)ovf_rep, ovf_cap, (unsigned long long*)ovf_counter};
  const int aligned = ((uintptr_t)text & 15) == 0;
  v3::launch_map3<v3::MAP_T, v3::MAP_SLOTS, v3::MAP_TPC>((const u8*)text, nbytes, rep_base, g, o, aligned, stream,
                                                          (u64*)stamps);
  hipLaunchKernelGGL(v3::ovf_agg3_kernel, dim3(1024), dim3(256), 0, stream, o, g);
  return (int)hipGetLastError();
}

}  // extern "C"
