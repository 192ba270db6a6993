// tail.hip — fused kernels of the reduce-side tail (compact -> partition ->
// (partition, key) sort -> key bytes -> download), the work that turns the
// HBM hash table into the sorted ``result.P<NN>`` columns (reference:
// job.lua:264-294 reduce + write, server.lua:346-411 result listing, SURVEY.md
// §2.2 K6/K8/K10/K11).
//
// The unfused tail was ~28 short launches; at small per-rank inputs (8-GPU
// strong scaling) the drain/fill between dependent kernels dominated.  Here:
//   compaction   : table -> dense rows + FNV-1 partition + composite sort key
//                  (part << 56 | hi >> 8) + the 8 digit histograms of that key
//                  (so the sort skips its histogram pass) + partition counts
//                  (mr_tail_compact: count / scatter / histogram launches);
//   [onesweep passes, sort.hip]
//   tail_gather  : rows reordered by the sort permutation + key lengths;
//   [tie fix-up, scan, key-byte gather: existing kernels]
//   tail_pack    : values, 32-bit offsets, partition counts and the fix-up
//                  flag packed into one buffer -> ONE device->host DMA.
#include <hip/hip_runtime.h>
#include "mr_common.h"
#include "hashtab.h"

namespace mr {
namespace tl {

constexpr int T = 256;


// Compaction of a table's occupied slots into dense rows, in launches sized
// for parallelism (one slot per thread; the first version gave each thread 4-16
// slots and one block-wide scan, so a 1 M-slot table ran ONE wave per SIMD:
// 50-73 us for 0.27 M keys, profiles/r2/tail):
//   tail_count_kernel   : occupied slots per block -> bcount[block]
//   tail_bscan_kernel   : one block: bcount -> exclusive block bases, and the
//                         row count (a per-block sum of its predecessors'
//                         counts was quadratic in the capacity: 33 us at 2^20
//                         slots, most of the scatter at 2^22-2^23)
//   tail_scatter_kernel : block base from the scan, wave ballots for the
//                         offsets inside the block, then the row (partition,
//                         composite key) of each slot
//   tail_hist_kernel    : the 8 digit histograms of the dense composite keys
//                         (and partition counts)
constexpr int CT = 512;  // compaction threads per block (one slot each)
constexpr int HIST_BLOCKS = 64;

// zero (optional): the tail's zeroed scratch (histograms, tile counters,
// flags), cleared by block 0 here instead of by a separate memset launch
// (everything that uses it runs after this kernel)
__global__ void __launch_bounds__(CT) tail_count_kernel(const GSlot* __restrict__ slots, u64 cap, u32* __restrict__ bcount,
                                                        u32* __restrict__ zero, u32 zwords) {
  __shared__ u32 wc[CT / 64];
  if (zero && blockIdx.x == 0)
    for (u32 k = threadIdx.x; k < zwords; k += CT) zero[k] = 0u;
  const u64 i = (u64)blockIdx.x * CT + threadIdx.x;
  const bool o = i < cap && slots[i].tag != 0;
  const u64 m = __ballot(o);
  if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = (u32)__popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) {
    u32 c = 0;
#pragma unroll
    for (int w = 0; w < CT / 64; ++w) c += wc[w];
    bcount[blockIdx.x] = c;
  }
}

constexpr int BS = 1024;  // threads of the block-count scan
__global__ void __launch_bounds__(BS) tail_bscan_kernel(u32* __restrict__ bcount, u64 nb,
                                                        unsigned long long* __restrict__ counter) {
  __shared__ u32 wsum[BS / 64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const u64 per = (nb + BS - 1) / BS;
  const u64 a = (u64)t * per, b = a + per < nb ? a + per : nb;
  u32 sum = 0;
  for (u64 j = a; j < b; ++j) sum += bcount[j];
  u32 incl = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const u32 y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  u32 base = 0, total = 0;
#pragma unroll
  for (int w = 0; w < BS / 64; ++w) {
    base += w < wave ? wsum[w] : 0u;
    total += wsum[w];
  }
  u32 run = base + incl - sum;
  for (u64 j = a; j < b; ++j) {
    const u32 c = bcount[j];
    bcount[j] = run;
    run += c;
  }
  if (t == 0) *counter = total;
}

__global__ void __launch_bounds__(CT) tail_scatter_kernel(GTab g, u64 cap, u32 nparts, const u8* __restrict__ src,
                                                          u64* __restrict__ out_hi, u64* __restrict__ out_lo,
                                                          long long* __restrict__ out_val, u64* __restrict__ out_rep,
                                                          u32* __restrict__ out_part, u64* __restrict__ out_c,
                                                          const u32* __restrict__ bbase, u64 out_cap) {
  __shared__ u32 wc[CT / 64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const u64 i = (u64)blockIdx.x * CT + t;
  const bool occ = i < cap && g.s[i].tag != 0;
  const u64 m = __ballot(occ);
  if (lane == 0) wc[wave] = (u32)__popcll(m);
  __syncthreads();
  u64 o = bbase[blockIdx.x];
#pragma unroll
  for (int w = 0; w < CT / 64; ++w) o += w < wave ? wc[w] : 0u;
  if (!occ) return;
  o += (u64)__popcll(m & ((1ull << lane) - 1ull));
  if (o >= out_cap) return;  // more rows than the caller's bound: flagged by tail_pad_kernel / the host
  const u64 h = g.s[i].hi, l = g.s[i].lo, r = g.s[i].rep;
  u32 len;
  const u32 f = key_fnv(h, l, r, src, &len);
  const u32 p = nparts ? f % nparts : f;
  out_hi[o] = h;
  out_lo[o] = l;
  out_val[o] = g.val[i];
  out_rep[o] = r;
  out_part[o] = p;
  out_c[o] = ((u64)p << 56) | (h >> 8);
}

// Rows [n, bound) of a compaction launched for a row BOUND instead of the
// host-known count (the W > 1 reduce tail: the count is never downloaded
// before the tail is queued).  They become sentinels that sort after every
// real row — composite key 0xFF << 56 | row, i.e. partition digit 0xFF, which
// no real row has when nparts <= 255, and distinct, so no tie run — with an
// empty key (hi = lo = 0: length 0) and a zero value.  The host takes the real
// count from the partition counts.  bad |= 8: the table had more rows than the
// bound (re-run with the count); bad |= 16: the table overflowed.
__global__ void tail_pad_kernel(const unsigned long long* __restrict__ counter, u64 bound, u64* __restrict__ out_hi,
                                u64* __restrict__ out_lo, long long* __restrict__ out_val, u64* __restrict__ out_rep,
                                u32* __restrict__ out_part, u64* __restrict__ out_c, const u32* __restrict__ ovf,
                                u32* __restrict__ bad) {
  const u64 n = *counter;
  const u64 stride = (u64)gridDim.x * blockDim.x;
  const u64 i0 = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (i0 == 0) {
    u32 b = n > bound ? 8u : 0u;
    if (ovf && *ovf) b |= 16u;
    if (b) atomicOr(bad, b);
  }
  for (u64 i = n + i0; i < bound; i += stride) {
    out_hi[i] = 0;
    out_lo[i] = 0;
    out_val[i] = 0;
    out_rep[i] = 0;
    out_part[i] = 0xFFu;
    out_c[i] = (0xFFull << 56) | i;
  }
}

// Digit histograms of the dense composite keys: LDS counts per block, then
// one global atomic per non-empty bin (few blocks: at most HIST_BLOCKS x 2048
// adds, each bin's chain HIST_BLOCKS long).  Digit 7 is the partition: its
// totals also go to pcount.
__global__ void __launch_bounds__(T) tail_hist_kernel(const u64* __restrict__ c, u64 n, u32* ghist, u32 nparts,
                                                      long long* pcount) {
  __shared__ u32 hist[8][256];
  const int t = threadIdx.x;
#pragma unroll
  for (int b = 0; b < 8; ++b) hist[b][t] = 0;
  __syncthreads();
  for (u64 i = (u64)blockIdx.x * T + t; i < n; i += (u64)gridDim.x * T) {
    const u64 x = c[i];
#pragma unroll
    for (int b = 0; b < 8; ++b) atomicAdd(&hist[b][(x >> (8 * b)) & 0xFF], 1u);
  }
  __syncthreads();
#pragma unroll
  for (int b = 0; b < 8; ++b)
    if (hist[b][t]) atomicAdd(&ghist[b * 256 + t], hist[b][t]);
  if (pcount && (u32)t < nparts && hist[7][t])
    atomicAdd((unsigned long long*)&pcount[t], (unsigned long long)hist[7][t]);
}

// Padded mode (a row BOUND): tail_pad_kernel and tail_hist_kernel in one
// launch — the sentinel rows [count, bound) are written and their composite
// keys histogrammed with the real ones (one launch less in the W > 1 tail).
// The block histograms are 16-bit counters, two per LDS word (4 KiB instead
// of 8: the kernel then fits beside the next map's workgroups, which leave
// 5 KiB of a CU's LDS), so a block may count at most 65535 rows (the caller
// checks).
__global__ void __launch_bounds__(T) tail_padhist_kernel(const unsigned long long* __restrict__ counter, u64 bound,
                                                         u64* __restrict__ out_hi, u64* __restrict__ out_lo,
                                                         long long* __restrict__ out_val, u64* __restrict__ out_rep,
                                                         u32* __restrict__ out_part, u64* __restrict__ out_c,
                                                         const u32* __restrict__ ovf, u32* __restrict__ bad,
                                                         u32* ghist, u32 nparts, long long* pcount) {
  __shared__ u32 hist[8][128];  // digit b, bin k: 16 bits at (k & 1) * 16 of word k >> 1
  const int t = threadIdx.x;
  if (t < 128)
#pragma unroll
    for (int b = 0; b < 8; ++b) hist[b][t] = 0;
  const u64 cnt = *counter;
  const u64 n = cnt < bound ? cnt : bound;
  if (blockIdx.x == 0 && t == 0) {
    u32 b = cnt > bound ? 8u : 0u;
    if (ovf && *ovf) b |= 16u;
    if (b) atomicOr(bad, b);
  }
  __syncthreads();
  for (u64 i = (u64)blockIdx.x * T + t; i < bound; i += (u64)gridDim.x * T) {
    u64 x;
    if (i < n) {
      x = out_c[i];
    } else {
      x = (0xFFull << 56) | i;
      out_hi[i] = 0;
      out_lo[i] = 0;
      out_val[i] = 0;
      out_rep[i] = 0;
      out_part[i] = 0xFFu;
      out_c[i] = x;
    }
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const u32 k = (u32)(x >> (8 * b)) & 0xFFu;
      atomicAdd(&hist[b][k >> 1], 1u << (16 * (k & 1u)));
    }
  }
  __syncthreads();
  const u32 sh = 16 * (t & 1);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const u32 c = (hist[b][t >> 1] >> sh) & 0xFFFFu;
    if (c) atomicAdd(&ghist[b * 256 + t], c);
    if (b == 7 && pcount && (u32)t < nparts && c) atomicAdd((unsigned long long*)&pcount[t], (unsigned long long)c);
  }
}

// Key offsets and key bytes of the sorted rows in one launch (the scan's
// apply step fused with the key-byte gather): block b takes rows
// [b * 4096, (b + 1) * 4096) (the scan's tiles; partials[b] = their base),
// 4 consecutive rows per thread; offs[i] = the exclusive prefix of the key
// lengths, and key i's bytes go to dst[offs[i] ..) (writes stop at dst_cap).
constexpr int OB_T = 1024, OB_ITEMS = 4;  // (256 x 16: 44.7 us vs 36.5 for the two launches)
__global__ void __launch_bounds__(OB_T) tail_offbytes_kernel(const long long* __restrict__ len, u64 n,
                                                             long long* __restrict__ offs,
                                                             const long long* __restrict__ partials,
                                                             const u64* __restrict__ hi, const u64* __restrict__ lo,
                                                             const u64* __restrict__ rep, const u8* __restrict__ src,
                                                             u8* __restrict__ dst, u64 dst_cap) {
  __shared__ long long wsum[OB_T / 64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const u64 my = (u64)blockIdx.x * OB_T * OB_ITEMS + (u64)t * OB_ITEMS;
  long long v[OB_ITEMS];
  long long sum = 0;
#pragma unroll
  for (int r = 0; r < OB_ITEMS; ++r) {
    v[r] = my + r < n ? len[my + r] : 0;
    sum += v[r];
  }
  long long incl = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const long long y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  long long off = partials[blockIdx.x] + incl - sum;
#pragma unroll
  for (int w = 0; w < OB_T / 64; ++w) off += w < wave ? wsum[w] : 0;
  for (int r = 0; r < OB_ITEMS; ++r) {
    const u64 i = my + r;
    if (i >= n) break;
    offs[i] = off;
    const u64 o = (u64)off;
    off += v[r];
    if (o >= dst_cap) continue;
    u8* d = dst + o;
    const u64 room = dst_cap - o;
    const u64 h = hi[i], l = lo[i];
    if (!key_is_long(l)) {
      const u32 kl = packed_len(l);
      for (u32 k = 0; k < kl && k < room; ++k) d[k] = (u8)packed_byte(h, l, k);
    } else {
      const u64 kl = rep_len(rep[i]) < room ? rep_len(rep[i]) : room;
      const u8* p = src + rep_off(rep[i]);
      copy_key_bytes(d, p, kl);
    }
  }
}

__global__ void tail_gather_kernel(const u32* __restrict__ perm, u64 n, const u64* __restrict__ hi,
                                   const u64* __restrict__ lo, const long long* __restrict__ val,
                                   const u64* __restrict__ rep, const u32* __restrict__ part, u64* __restrict__ o_hi,
                                   u64* __restrict__ o_lo, long long* __restrict__ o_val, u64* __restrict__ o_rep,
                                   u32* __restrict__ o_part, long long* __restrict__ o_len) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const u64 j = clamp_row(perm[i], n);
    const u64 l = lo[j], r = rep[j];
    o_hi[i] = hi[j];
    o_lo[i] = l;
    o_val[i] = val[j];
    o_rep[i] = r;
    o_part[i] = part[j];
    o_len[i] = key_is_long(l) ? (long long)rep_len(r) : (long long)packed_len(l);
  }
}

// [val: n x i64][off: (n+1) x i32][counts: nparts x i64][bad: u32] (8-byte aligned sections)
// bad: bit 0 = a tie run too long for the fixup, bit 1 = unchecked long-key
// prefix tie, bit 2 = the sort's decoupled look-back gave up (`err`: the
// order is wrong; the host re-sorts or raises)
__global__ void tail_pack_kernel(const long long* __restrict__ val, const long long* __restrict__ off, u64 n,
                                 const long long* __restrict__ counts, u32 nparts, const u32* __restrict__ bad,
                                 const u32* __restrict__ err, u8* __restrict__ out) {
  long long* ov = (long long*)out;
  int* oo = (int*)(out + 8 * n);
  const u64 off_bytes = ((4 * (n + 1)) + 7) & ~7ull;
  long long* oc = (long long*)(out + 8 * n + off_bytes);
  u32* ob = (u32*)(out + 8 * n + off_bytes + 8 * (u64)nparts);
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += stride) {
    if (i < n) ov[i] = val[i];
    oo[i] = (int)off[i];
    if (i < nparts) oc[i] = counts[i];
    if (i == 0) ob[0] = bad[0] | ((err && err[0]) ? 4u : 0u);
  }
  if (blockIdx.x == 0 && threadIdx.x < nparts && n + 1 <= threadIdx.x) oc[threadIdx.x] = counts[threadIdx.x];
}

}  // namespace tl
}  // namespace mr

using namespace mr;

extern "C" {

u64 mr_tail_pack_bytes(u64 n, u32 nparts) { return 8 * n + (((4 * (n + 1)) + 7) & ~7ull) + 8 * (u64)nparts + 8; }

// Bytes of the compaction scratch (`bhist`) of mr_tail_compact: per-block
// slot counts.
u64 mr_tail_bhist_bytes(u64 cap) { return ((cap + tl::CT - 1) / tl::CT * 4 + 255) & ~255ull; }

// Occupied slots -> dense rows (+ partition, composite key).  With ghist: its
// 8 digit histograms (+ partition counts into pcount); n = the number of
// occupied slots (host-known: it sizes the histogram grid).
// out_cap: rows the outputs hold (slots past it are dropped; the count in
// `counter` still says how many there were).  pad != 0: n is a row BOUND, the
// rows [count, n) become sentinels (tail_pad_kernel; nparts <= 255) and the
// histograms cover all n rows; `bad` gets the bound / overflow flags.
static int tail_compact(void* tag, void* hi, void* lo, void* val, void* rep, void* ctrl, u64 cap, u32 nparts,
                        const void* src, void* out_hi, void* out_lo, void* out_val, void* out_rep, void* out_part,
                        void* out_c, void* counter, void* ghist, void* pcount, void* bhist, u64 n, u64 out_cap, int pad,
                        void* bad, void* zero, u32 zbytes, hipStream_t s);

int mr_tail_compact(void* tag, void* hi, void* lo, void* val, void* rep, void* ctrl, u64 cap, u32 nparts,
                    const void* src, void* out_hi, void* out_lo, void* out_val, void* out_rep, void* out_part,
                    void* out_c, void* counter, void* ghist, void* pcount, void* bhist, u64 n, u64 out_cap, int pad,
                    void* bad, hipStream_t s) {
  return tail_compact(tag, hi, lo, val, rep, ctrl, cap, nparts, src, out_hi, out_lo, out_val, out_rep, out_part, out_c,
                      counter, ghist, pcount, bhist, n, out_cap, pad, bad, nullptr, 0, s);
}

}  // extern "C"

static int tail_compact(void* tag, void* hi, void* lo, void* val, void* rep, void* ctrl, u64 cap, u32 nparts,
                        const void* src, void* out_hi, void* out_lo, void* out_val, void* out_rep, void* out_part,
                        void* out_c, void* counter, void* ghist, void* pcount, void* bhist, u64 n, u64 out_cap, int pad,
                        void* bad, void* zero, u32 zbytes, hipStream_t s) {
  if (nparts > 256 || bhist == nullptr || (pad && (nparts > 255 || bad == nullptr))) return -1;
  GTab g = gtab_make(tag, val, ctrl, cap, nullptr);
  const u64 nb = (cap + tl::CT - 1) / tl::CT;
  u32* bcount = (u32*)bhist;
  hipLaunchKernelGGL(tl::tail_count_kernel, dim3((unsigned)nb), dim3(tl::CT), 0, s, (const GSlot*)tag, cap, bcount,
                     (u32*)zero, zbytes / 4);
  hipLaunchKernelGGL(tl::tail_bscan_kernel, dim3(1), dim3(tl::BS), 0, s, bcount, nb, (unsigned long long*)counter);
  hipLaunchKernelGGL(tl::tail_scatter_kernel, dim3((unsigned)nb), dim3(tl::CT), 0, s, g, cap, nparts, (const u8*)src,
                     (u64*)out_hi, (u64*)out_lo, (long long*)out_val, (u64*)out_rep, (u32*)out_part, (u64*)out_c,
                     (const u32*)bcount, out_cap);
  u64 phb = (n + 4 * tl::T - 1) / (4 * tl::T);
  if (phb > (u64)tl::HIST_BLOCKS) phb = tl::HIST_BLOCKS;
  // 16-bit counters: a block walks ceil(n / (hb * T)) grid strides of T rows,
  // all of which may fall in one bin — that must stay <= 65535 (a bound on the
  // rows per BLOCK, not on the total: the grid is capped at HIST_BLOCKS)
  const u64 rows_per_block = phb ? (n + phb * tl::T - 1) / (phb * tl::T) * tl::T : 0;
  if (pad && n > 0 && ghist != nullptr && rows_per_block <= 65535u) {
    const u64 hb = phb;
    hipLaunchKernelGGL(tl::tail_padhist_kernel, dim3((unsigned)hb), dim3(tl::T), 0, s, (const unsigned long long*)counter,
                       n, (u64*)out_hi, (u64*)out_lo, (long long*)out_val, (u64*)out_rep, (u32*)out_part, (u64*)out_c,
                       (const u32*)ctrl + 1, (u32*)bad, (u32*)ghist, nparts, (long long*)pcount);
    return (int)hipGetLastError();
  }
  if (pad && n > 0) {
    u64 pb = (n + 255) / 256;
    if (pb > 1024) pb = 1024;
    hipLaunchKernelGGL(tl::tail_pad_kernel, dim3((unsigned)pb), dim3(256), 0, s, (const unsigned long long*)counter, n,
                       (u64*)out_hi, (u64*)out_lo, (long long*)out_val, (u64*)out_rep, (u32*)out_part, (u64*)out_c,
                       (const u32*)ctrl + 1, (u32*)bad);
  }
  if (ghist != nullptr && n > 0) {
    u64 hb = (n + 4 * tl::T - 1) / (4 * tl::T);
    if (hb > (u64)tl::HIST_BLOCKS) hb = tl::HIST_BLOCKS;
    hipLaunchKernelGGL(tl::tail_hist_kernel, dim3((unsigned)hb), dim3(tl::T), 0, s, (const u64*)out_c, n, (u32*)ghist,
                       nparts, (long long*)pcount);
  }
  return (int)hipGetLastError();
}

extern "C" {

int mr_tail_gather(const void* perm, u64 n, const void* hi, const void* lo, const void* val, const void* rep,
                   const void* part, void* o_hi, void* o_lo, void* o_val, void* o_rep, void* o_part, void* o_len,
                   hipStream_t s) {
  if (n == 0) return 0;
  u64 g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(tl::tail_gather_kernel, dim3((unsigned)g), dim3(256), 0, s, (const u32*)perm, n, (const u64*)hi,
                     (const u64*)lo, (const long long*)val, (const u64*)rep, (const u32*)part, (u64*)o_hi,
                     (u64*)o_lo, (long long*)o_val, (u64*)o_rep, (u32*)o_part, (long long*)o_len);
  return (int)hipGetLastError();
}

int mr_tail_pack(const void* val, const void* off, u64 n, const void* counts, u32 nparts, const void* bad,
                 const void* err, void* out, hipStream_t s) {
  if (nparts > 256) return -1;
  u64 g = (n + 1 + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(tl::tail_pack_kernel, dim3((unsigned)g), dim3(256), 0, s, (const long long*)val,
                     (const long long*)off, n, (const long long*)counts, nparts, (const u32*)bad, (const u32*)err,
                     (u8*)out);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// The whole fused tail in ONE host call: every launch and both downloads are
// queued from C++ instead of ~20 Python-level calls and tensor allocations per
// iteration (at 8-GPU strong scaling the per-iteration host time was a large
// part of the ~1 ms step).  All buffers live in one caller-owned workspace
// (layout below, mr_tail_ws_layout), reused across iterations — except the
// decoupled-look-back granules of its sort, which have a buffer of their own
// (own epoch counter; see mr_tail_run).

int mr_exclusive_scan_i64(const void* in, void* out, u64 n, void* partials, void* total, hipStream_t s);
u64 mr_scan_partials_len(u64 n);
u64 mr_scan_tile();
int mr_scan_partials_i64(const void* in, u64 n, void* partials, void* total, hipStream_t s);
u64 mr_onesweep_tiles(u64 n);
int mr_radix_onesweep_u32v(const void* keys_in, const void* vals_in, void* keys_out, void* vals_out, u64 n, int shift,
                           const void* ghist, void* granules, void* tile_counter, u32 epoch, void* err, int iota,
                           hipStream_t s);
int mr_tie_fixup(const void* c, void* hi, void* lo, void* val, void* rep, void* part, u64 n, void* bad,
                 const void* src, void* ln, hipStream_t s);
int mr_gather_key_bytes(const void* hi, const void* lo, const void* rep, const void* off, u64 n, const void* src,
                        void* dst, u64 dst_cap, hipStream_t stream);
int mr_copy_to_host(const void* src, void* host_dst, const void* nelem, u64 elem_size, u64 max_bytes, hipStream_t s);
int mr_d2h_async(void* host_dst, const void* src, u64 nbytes, hipStream_t s);

enum TailBuf : int {
  TB_HI0, TB_LO0, TB_VAL0, TB_REP0, TB_C, TB_PART0, TB_ZERO /* counter|ghist|pcount|sort ctrs|err|bad */,
  TB_K0, TB_K1, TB_P0, TB_P1, TB_HI, TB_LO, TB_VAL, TB_REP, TB_PART, TB_LN, TB_OFF, TB_PARTIALS,
  TB_BLOB, TB_PACKED, TB_BHIST, TB_COUNT
};
// TB_ZERO sub-layout (bytes): counter u64 @0 | ghist u32[2048] @8 | pcount i64[256] @8200 |
// sort tile counters u32[64] @10248 | sort err u32 @10504 | bad u32 @10508
constexpr u64 TZ_GHIST = 8, TZ_PCOUNT = 8200, TZ_TILES = 10248, TZ_ERR = 10504, TZ_BAD = 10508, TZ_BYTES = 10512;

u64 mr_tail_ws_layout(u64 n, u32 nparts, u64 blob_cap, u64 cap, u64* off) {
  (void)nparts;
  const u64 m = n ? n : 1;
  const u64 sz[TB_COUNT] = {8 * m, 8 * m, 8 * m, 8 * m, 8 * m, 4 * m, TZ_BYTES, 8 * m, 8 * m, 4 * m, 4 * m,
                            8 * m, 8 * m, 8 * m, 8 * m, 4 * m, 8 * m, 8 * (m + 1),
                            8 * mr_scan_partials_len(m), blob_cap ? blob_cap : 1, mr_tail_pack_bytes(m, 256),
                            mr_tail_bhist_bytes(cap)};
  u64 o = 0;
  for (int i = 0; i < TB_COUNT; ++i) {
    off[i] = o;
    o += (sz[i] + 255) & ~255ull;
  }
  return o;
}

static u32 g_tail_epoch = 0;

// n = occupied slots of the table; src = the key-byte source (map arena or the
// received blob); hp / hb = pinned host buffers of the packed columns and the
// key bytes; est >= 0: DMA min(est, hb_cap) key bytes, else a device-sized copy.
// padded != 0: n is a row bound, not the count (tail_pad_kernel): the host
// learns the count from the downloaded partition counts, and bits 3/4 of the
// downloaded flag word if the bound was too small / the table overflowed.
// gran: the sort's look-back granules, >= 256 * mr_onesweep_tiles(n) u64 of a
// buffer that holds nothing else (zeroed when allocated).  They used to be a
// region of ws, whose layout moves with n: a later tail's granule rows then lay
// over an earlier tail's permutation words, whose top bits can read as a live
// epoch tag — a late predecessor's granule was taken from that stale word and
// the pass scattered with a wrong prefix, silently (seen with 4 worker
// processes sharing one GPU, whose contention makes predecessors late, and
// whose fresh processes run small epochs; profiles/r6/server_worker/).
int mr_tail_run(void* tag, void* hi, void* lo, void* val, void* rep, void* ctrl, u64 cap, u64 n, u32 nparts,
                const void* src, void* ws, void* gran, u64 blob_cap, void* hp, void* hb, long long est, u64 hb_cap,
                int padded, hipStream_t s) {
  if (gran == nullptr) return -1;
  if (nparts > 256 || (padded && nparts > 255)) return -1;
  u64 off[TB_COUNT];
  mr_tail_ws_layout(n, nparts, blob_cap, cap, off);
  u8* w = (u8*)ws;
  auto P = [&](int b) { return (void*)(w + off[b]); };
  u8* z = w + off[TB_ZERO];
  // (the zeroed scratch z is cleared by the compaction's first kernel)
  int rc = tail_compact(tag, hi, lo, val, rep, ctrl, cap, nparts, src, P(TB_HI0), P(TB_LO0), P(TB_VAL0), P(TB_REP0),
                        P(TB_PART0), P(TB_C), z, z + TZ_GHIST, z + TZ_PCOUNT, P(TB_BHIST), n, n, padded, z + TZ_BAD,
                        z, (u32)TZ_BYTES, s);
  if (rc) return rc;
  // 8 onesweep passes over the composite key (ghist from tail_compact)
  const void* kin = P(TB_C);
  const void* pin = nullptr;
  for (int pass = 0; pass < 8; ++pass) {
    g_tail_epoch = (g_tail_epoch + 1) & 0xFFFFFFu;
    if (!g_tail_epoch) g_tail_epoch = 1;
    void* kout = P(pass & 1 ? TB_K1 : TB_K0);
    void* pout = P(pass & 1 ? TB_P1 : TB_P0);
    rc = mr_radix_onesweep_u32v(kin, pin, kout, pout, n, 8 * pass, z + TZ_GHIST + 4 * 256 * pass, gran,
                                z + TZ_TILES + 4 * pass, g_tail_epoch, z + TZ_ERR, pass == 0 ? 1 : 0, s);
    if (rc) return rc;
    kin = kout;
    pin = pout;
  }
  rc = mr_tail_gather(pin, n, P(TB_HI0), P(TB_LO0), P(TB_VAL0), P(TB_REP0), P(TB_PART0), P(TB_HI), P(TB_LO),
                      P(TB_VAL), P(TB_REP), P(TB_PART), P(TB_LN), s);
  if (rc) return rc;
  rc = mr_tie_fixup(kin, P(TB_HI), P(TB_LO), P(TB_VAL), P(TB_REP), P(TB_PART), n, z + TZ_BAD, src, P(TB_LN), s);
  if (rc) return rc;
  long long* offs = (long long*)P(TB_OFF);
  if (n > 16384 && mr_scan_tile() == (u64)tl::OB_T * tl::OB_ITEMS) {
    // tile sums + their scan, then offsets and key bytes in one launch
    rc = mr_scan_partials_i64(P(TB_LN), n, P(TB_PARTIALS), offs + n, s);
    if (rc) return rc;
    const u64 nt = (n + mr_scan_tile() - 1) / mr_scan_tile();
    hipLaunchKernelGGL(tl::tail_offbytes_kernel, dim3((unsigned)nt), dim3(tl::OB_T), 0, s, (const long long*)P(TB_LN),
                       n, offs, (const long long*)P(TB_PARTIALS), (const u64*)P(TB_HI), (const u64*)P(TB_LO),
                       (const u64*)P(TB_REP), (const u8*)src, (u8*)P(TB_BLOB), blob_cap ? blob_cap : 1);
    rc = (int)hipGetLastError();
  } else {
    if (n) {
      rc = mr_exclusive_scan_i64(P(TB_LN), offs, n, P(TB_PARTIALS), offs + n, s);
    } else {
      rc = (int)hipMemsetAsync(offs, 0, 8, s);
    }
    if (rc) return rc;
    rc = mr_gather_key_bytes(P(TB_HI), P(TB_LO), P(TB_REP), offs, n, src, P(TB_BLOB), blob_cap ? blob_cap : 1, s);
  }
  if (rc) return rc;
  rc = mr_tail_pack(P(TB_VAL), offs, n, z + TZ_PCOUNT, nparts, z + TZ_BAD, z + TZ_ERR, P(TB_PACKED), s);
  if (rc) return rc;
  rc = mr_d2h_async(hp, P(TB_PACKED), mr_tail_pack_bytes(n, nparts), s);
  if (rc) return rc;
  if (est >= 0) {
    const u64 nb = (u64)est < hb_cap ? (u64)est : hb_cap;
    if (nb) rc = mr_d2h_async(hb, P(TB_BLOB), nb < blob_cap ? nb : blob_cap, s);
  } else {
    rc = mr_copy_to_host(P(TB_BLOB), hb, offs + n, 1, hb_cap, s);
  }
  return rc;
}

}  // extern "C"
