// shuffle.hip — pack a rank's combined (key, value) table by destination rank
// for the all-to-all shuffle (reference: the per-partition map_results files
// job.lua:203-221 and their transport), and fix up the
// received key locations.
//
// One record per distinct key: [hi, lo, val, loc] where loc = (byte offset in
// the destination's key-byte segment) << 24 | key length.  Key bytes of every
// record are packed into per-destination contiguous segments, so the payload
// is two all_to_all_single calls (records, bytes) after one count exchange.
// Records and bytes are placed with per-workgroup range reservations (one
// global atomic per (workgroup, destination)), so there is no sort by
// destination and no separate gather: order inside a destination segment is
// irrelevant because the receiver re-aggregates by key.
//
//   pk_count   : per-destination record and byte counts
//   pk_scan    : exclusive scans -> segment starts; counts -> exchange buffer
//   pk_scatter : records + key bytes into their segments
//   pk_fix_loc : received loc -> absolute (offset in the received byte blob)
#include <hip/hip_runtime.h>
#include "mr_common.h"
#include "hashtab.h"

namespace mr {
namespace pk {

constexpr int T = 256;
constexpr int MAXW = 256;

__device__ __forceinline__ u32 key_len(u64 lo, u64 rep) { return key_is_long(lo) ? (u32)rep_len(rep) : packed_len(lo); }

__global__ void __launch_bounds__(T) pk_count_kernel(const u64* __restrict__ lo, const u64* __restrict__ rep,
                                                     const u32* __restrict__ part, u64 n, u32 W,
                                                     unsigned long long* __restrict__ cnt /*[2W]*/) {
  __shared__ u32 rc[MAXW];
  __shared__ unsigned long long bc[MAXW];
  for (u32 d = threadIdx.x; d < W; d += T) {
    rc[d] = 0;
    bc[d] = 0;
  }
  __syncthreads();
  const u64 stride = (u64)gridDim.x * T;
  for (u64 i = (u64)blockIdx.x * T + threadIdx.x; i < n; i += stride) {
    const u32 d = part[i] % W;
    atomicAdd(&rc[d], 1u);
    atomicAdd(&bc[d], (unsigned long long)key_len(lo[i], rep[i]));
  }
  __syncthreads();
  for (u32 d = threadIdx.x; d < W; d += T) {
    if (rc[d]) atomicAdd(&cnt[d], (unsigned long long)rc[d]);
    if (bc[d]) atomicAdd(&cnt[W + d], bc[d]);
  }
}

// Bytes of destination/source d's segment in the combined layout: its
// records (32 B each), then its key bytes padded to 8.
__host__ __device__ __forceinline__ u64 seg_bytes(u64 rows, u64 bytes) { return 32 * rows + ((bytes + 7) & ~7ull); }

// cnt [2W] -> start [2W] = BYTE offsets of destination d's records (start[d])
// and key bytes (start[W+d]), cursors zeroed, and the exchange row per
// destination: xchg[3d] = records, xchg[3d+1] = bytes, xchg[3d+2] = extra.
// Separate layout: records in one array, key bytes in another.  Combined
// layout: ONE buffer of per-destination segments [records | key bytes], so
// the payload is a single all_to_all_single.
//
// Status (the W > 1 single-sync iteration, cp_scatter_kernel below): the map's
// completion checks ride on the count exchange instead of a host read before
// it.  If the map table overflowed, a map chunk set its error word or the send
// buffer is too small, extra gets STATUS_REDO added: every rank sees it in the
// exchanged counts and the exchange is redone after the flagged rank fixed its
// map (or grew its buffer to the exchanged totals).
constexpr long long STATUS_REDO = 1ll << 40;
__global__ void pk_scan_kernel(const unsigned long long* __restrict__ cnt, u32 W, unsigned long long* __restrict__ start,
                               unsigned long long* __restrict__ cursor, long long* __restrict__ xchg, long long extra,
                               int combined) {
  if (threadIdx.x != 0) return;
  unsigned long long r = 0, b = 0;
  for (u32 d = 0; d < W; ++d) {
    if (combined) {
      start[d] = r;
      start[W + d] = r + 32 * cnt[d];
      r += seg_bytes(cnt[d], cnt[W + d]);
    } else {
      start[d] = 32 * r;
      start[W + d] = b;
      r += cnt[d];
      b += cnt[W + d];
    }
    cursor[d] = 0;
    cursor[W + d] = 0;
    xchg[3 * d] = (long long)cnt[d];
    xchg[3 * d + 1] = (long long)cnt[W + d];
    xchg[3 * d + 2] = extra;
  }
}

__global__ void __launch_bounds__(T) pk_scatter_kernel(const u64* __restrict__ hi, const u64* __restrict__ lo,
                                                       const long long* __restrict__ val, const u64* __restrict__ rep,
                                                       const u32* __restrict__ part, u64 n, u32 W,
                                                       const u8* __restrict__ src,
                                                       const unsigned long long* __restrict__ start,
                                                       unsigned long long* __restrict__ cursor,
                                                       u8* __restrict__ rec /*records, byte-addressed*/,
                                                       u8* __restrict__ blob) {
  __shared__ u32 rc[MAXW];
  __shared__ u32 bc[MAXW];
  __shared__ unsigned long long rbase[MAXW];
  __shared__ unsigned long long bbase[MAXW];
  const u64 i = (u64)blockIdx.x * T + threadIdx.x;
  for (u32 d = threadIdx.x; d < W; d += T) {
    rc[d] = 0;
    bc[d] = 0;
  }
  __syncthreads();
  u32 d = 0, len = 0, rpos = 0, bpos = 0;
  const bool live = i < n;
  if (live) {
    d = part[i] % W;
    len = key_len(lo[i], rep[i]);
    rpos = atomicAdd(&rc[d], 1u);
    bpos = atomicAdd(&bc[d], len);
  }
  __syncthreads();
  for (u32 k = threadIdx.x; k < W; k += T) {
    rbase[k] = rc[k] ? atomicAdd(&cursor[k], (unsigned long long)rc[k]) : 0;
    bbase[k] = bc[k] ? atomicAdd(&cursor[W + k], (unsigned long long)bc[k]) : 0;
  }
  __syncthreads();
  if (!live) return;
  u64* rr = reinterpret_cast<u64*>(rec + start[d] + 32 * (rbase[d] + rpos));
  const u64 boff = bbase[d] + bpos;  // offset inside destination d's byte segment
  const u64 h = hi[i], l = lo[i];
  rr[0] = h;
  rr[1] = l;
  rr[2] = (u64)val[i];
  rr[3] = make_rep(boff, len);
  u8* out = blob + start[W + d] + boff;
  if (!key_is_long(l)) {
    for (u32 k = 0; k < len; ++k) out[k] = (u8)packed_byte(h, l, k);
  } else {
    const u8* p = src + rep_off(rep[i]);
    copy_key_bytes(out, p, len);
  }
}

// ---------------------------------------------------------------------------
// Send side straight from the map's hash table (the W > 1 single-sync
// iteration): three launches instead of the compaction's three plus the
// pack's four, and no dense intermediate columns.
//   cp_count   : per table block (CP * CP_PER = 512 slots, one per thread), per
//                destination, the rows and key bytes of its occupied slots ->
//                bcnt[2W][block] (u64: the exclusive bases of the byte columns
//                reach 4 GiB for a destination of large key sets)
//   cp_scan    : one workgroup per (destination, rows | bytes) column: the
//                exclusive prefix over the blocks and the column's total
//   cp_scatter : (block 0) segment starts, the count-exchange row and the
//                status (table overflow, chunk errors, send buffer too small)
//                then each slot again -> its record + key bytes at the block's
//                base in its destination's segment (LDS-atomic ranks inside
//                the block: order inside a segment is irrelevant, the
//                receiver re-aggregates by key)
constexpr int CP = 512;       // threads per block
constexpr int CP_PER = 1;     // table slots per thread (8: 4096-slot blocks ran cp_count / cp_scatter 2x slower)

__device__ __forceinline__ bool cp_slot(const GTab& g, u64 cap, u64 i, u32 nparts, u32 W, const u8* src, u64& h,
                                        u64& l, u64& r, u32& d, u32& len) {
  if (i >= cap || g.s[i].tag == 0) return false;
  h = g.s[i].hi;
  l = g.s[i].lo;
  r = g.s[i].rep;
  const u32 f = key_fnv(h, l, r, src, &len);
  d = (nparts ? f % nparts : f) % W;
  return true;
}

__global__ void __launch_bounds__(CP) cp_count_kernel(GTab g, u64 cap, u32 nparts, u32 W, const u8* __restrict__ src,
                                                      unsigned long long* __restrict__ bcnt) {
  __shared__ u32 rc[MAXW], bc[MAXW];
  for (u32 k = threadIdx.x; k < W; k += CP) rc[k] = bc[k] = 0;
  __syncthreads();
  const u64 i0 = (u64)blockIdx.x * CP * CP_PER + threadIdx.x;
#pragma unroll
  for (int it = 0; it < CP_PER; ++it) {
    u64 h, l, r;
    u32 d, len;
    if (cp_slot(g, cap, i0 + (u64)it * CP, nparts, W, src, h, l, r, d, len)) {
      atomicAdd(&rc[d], 1u);
      atomicAdd(&bc[d], len);
    }
  }
  __syncthreads();
  const u64 nb = gridDim.x;  // column-major [2W][nb]: a column's blocks are contiguous for the scan
  for (u32 k = threadIdx.x; k < W; k += CP) {
    bcnt[(u64)k * nb + blockIdx.x] = rc[k];
    bcnt[(u64)(W + k) * nb + blockIdx.x] = bc[k];
  }
}

// One workgroup per column of bcnt ([2W][nb], column-major): the exclusive
// prefix of the column over the blocks, written back in place, and the
// column's total into coltot[c].  Thread t owns the blocks
// [t * per, (t + 1) * per), read CS_K at a time with their loads issued
// together.  (A single 1024-thread workgroup for all columns took 50-63 us:
// it waited for a CU beside the map's workgroups and walked its blocks
// serially.)
constexpr int CS = 256;
constexpr int CS_K = 8;
__global__ void __launch_bounds__(CS) cp_scan_kernel(unsigned long long* __restrict__ bcnt, u64 nb,
                                                     unsigned long long* __restrict__ coltot) {
  __shared__ unsigned long long ws[CS / 64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  unsigned long long* col = bcnt + (u64)blockIdx.x * nb;
  const u64 per = (nb + CS - 1) / CS;
  const u64 a = (u64)t * per < nb ? (u64)t * per : nb, b = a + per < nb ? a + per : nb;
  unsigned long long sum = 0;
  for (u64 j = a; j < b; j += CS_K) {
    unsigned long long v[CS_K];
#pragma unroll
    for (int k = 0; k < CS_K; ++k) v[k] = j + k < b ? col[j + k] : 0ull;
#pragma unroll
    for (int k = 0; k < CS_K; ++k) sum += v[k];
  }
  unsigned long long incl = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) ws[wave] = incl;
  __syncthreads();
  unsigned long long run = incl - sum, all = 0;
#pragma unroll
  for (int w = 0; w < CS / 64; ++w) {
    run += w < wave ? ws[w] : 0ull;
    all += ws[w];
  }
  for (u64 j = a; j < b; j += CS_K) {
    unsigned long long v[CS_K];
#pragma unroll
    for (int k = 0; k < CS_K; ++k) v[k] = j + k < b ? col[j + k] : 0ull;
#pragma unroll
    for (int k = 0; k < CS_K; ++k) {
      if (j + k < b) col[j + k] = run;  // exclusive base of block j + k
      run += v[k];
    }
  }
  if (t == 0) coltot[blockIdx.x] = all;
}

__global__ void __launch_bounds__(CP) cp_scatter_kernel(GTab g, u64 cap, u32 nparts, u32 W, const u8* __restrict__ src,
                                                        const unsigned long long* __restrict__ bcnt,
                                                        const unsigned long long* __restrict__ coltot,
                                                        u8* __restrict__ buf, u64 buf_cap, long long* __restrict__ xchg,
                                                        long long extra, const u32* __restrict__ ovf,
                                                        const int* __restrict__ errs, u32 nerr,
                                                        unsigned long long* __restrict__ rows_out) {
  __shared__ u32 rc[MAXW], bc[MAXW];
  extern __shared__ unsigned long long start[];  // [2W]: destination d's records, then its key bytes
  for (u32 k = threadIdx.x; k < W; k += CP) rc[k] = bc[k] = 0;
  if (threadIdx.x == 0) {
    unsigned long long off = 0, rows = 0;
    for (u32 d = 0; d < W; ++d) {
      start[d] = off;
      start[W + d] = off + 32 * coltot[d];
      off += seg_bytes(coltot[d], coltot[W + d]);
      rows += coltot[d];
    }
    if (blockIdx.x == 0) {
      // the count-exchange row and the status (the map's checks, a send
      // buffer too small for the segments: the exchange is redone)
      bool redo = (ovf && *ovf) || off > buf_cap;
      for (u32 k = 0; errs && k < nerr; ++k) redo |= errs[k] != 0;
      for (u32 d = 0; d < W; ++d) {
        xchg[3 * d] = (long long)coltot[d];
        xchg[3 * d + 1] = (long long)coltot[W + d];
        xchg[3 * d + 2] = extra + (redo ? STATUS_REDO : 0);
      }
      *rows_out = rows;
    }
  }
  __syncthreads();
  const u64 nb = gridDim.x;
  const u64 i0 = (u64)blockIdx.x * CP * CP_PER + threadIdx.x;
  for (int it = 0; it < CP_PER; ++it) {
    const u64 i = i0 + (u64)it * CP;
    u64 h = 0, l = 0, r = 0;
    u32 d = 0, len = 0;
    if (!cp_slot(g, cap, i, nparts, W, src, h, l, r, d, len)) continue;
    const u32 rpos = atomicAdd(&rc[d], 1u);
    const u32 bpos = atomicAdd(&bc[d], len);
    const u64 ro = start[d] + 32 * (bcnt[(u64)d * nb + blockIdx.x] + rpos);
    const u64 boff = bcnt[(u64)(W + d) * nb + blockIdx.x] + bpos;  // inside destination d's byte segment
    const u64 bo = start[W + d] + boff;
    if (ro + 32 > buf_cap || bo + len > buf_cap) continue;  // too small: flagged by block 0 above, the exchange is redone
    u64* rr = reinterpret_cast<u64*>(buf + ro);
    rr[0] = h;
    rr[1] = l;
    rr[2] = (u64)g.val[i];
    rr[3] = make_rep(boff, len);
    u8* out = buf + bo;
    if (!key_is_long(l)) {
      for (u32 k = 0; k < len; ++k) out[k] = (u8)packed_byte(h, l, k);
    } else {
      const u8* p = src + rep_off(r);
      copy_key_bytes(out, p, len);
    }
  }
}

// Received records from source s carry offsets relative to s's byte segment;
// make them absolute: loc += byte_start(s) << 24, s found from the record
// prefix counts (rstart[W+1] / bstart[W] on the device).
__global__ void pk_fix_loc_kernel(u64* __restrict__ rec, u64 n, const long long* __restrict__ rstart,
                                  const long long* __restrict__ bstart, u32 W, u64* __restrict__ rep_out) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    u32 a = 0, b = W;  // source s: rstart[s] <= i < rstart[s+1]
    while (b - a > 1) {
      const u32 m = (a + b) >> 1;
      if ((long long)i >= rstart[m]) a = m;
      else b = m;
    }
    const u64 loc = rec[4 * i + 3];
    rep_out[i] = make_rep(rep_off(loc) + (u64)bstart[a], rep_len(loc));
  }
}

// Receive side in ONE launch: records [hi, lo, val, loc] from W sources (row
// and byte counts per source in `recv` = the count-exchange row [W][3] on the
// device) are folded into the reduce table with absolute rep words (loc made
// relative to the received byte blob).  Replaces the column splits, the
// host-built prefix arrays and their H2D copies, fix_loc and hash_agg.
constexpr int MAXW_RECV = 1024;
__global__ void __launch_bounds__(256) pk_insert_received_kernel(const u8* __restrict__ rec, u64 n,
                                                                 const long long* __restrict__ recv, u32 W, GTab g,
                                                                 int op, int combined) {
  // LDS sized by W at launch (3 (W + 1) words: ~200 B at W = 8, not the 24 KiB
  // of MAXW_RECV-sized arrays): the insert then fits beside the next map's
  // workgroups (77.5 KiB each, two per CU) instead of waiting for one to retire
  extern __shared__ long long pk_lds[];
  long long* rstart = pk_lds;              // first row of source k
  long long* rbyte = rstart + (W + 1);     // byte offset of source k's records
  long long* bstart = rbyte + (W + 1);     // byte offset of source k's key bytes
  if (threadIdx.x == 0) {  // W is small (ranks of one job): a serial prefix sum
    long long r = 0, b = 0, seg = 0;
    for (u32 k = 0; k < W; ++k) {
      rstart[k] = r;
      if (combined) {
        rbyte[k] = seg;
        bstart[k] = seg + 32 * recv[3 * k];
        seg += (long long)seg_bytes((u64)recv[3 * k], (u64)recv[3 * k + 1]);
      } else {
        rbyte[k] = 32 * r;
        bstart[k] = b;
      }
      r += recv[3 * k];
      b += recv[3 * k + 1];
    }
    rstart[W] = r;
    bstart[W] = b;
  }
  __syncthreads();
  const u64 stride = (u64)gridDim.x * blockDim.x;
  u32 claims = 0;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    u32 a = 0, b = W;
    while (b - a > 1) {
      const u32 m = (a + b) >> 1;
      if ((long long)i >= rstart[m]) a = m;
      else b = m;
    }
    const u64* r = reinterpret_cast<const u64*>(rec + rbyte[a] + 32 * (i - (u64)rstart[a]));
    const u64 loc = r[3];
    const u64 rep = make_rep(rep_off(loc) + (u64)bstart[a], rep_len(loc));
    claims += gtab_insert(g, r[0], r[1], (long long)r[2], rep, op) == 2;
  }
  gtab_count_claims(g, claims);
}

}  // namespace pk
}  // namespace mr

using namespace mr;

static inline unsigned pk_grid(u64 n, unsigned cap = 4096) {
  u64 g = (n + pk::T - 1) / pk::T;
  return (unsigned)(g < 1 ? 1 : (g > cap ? cap : g));
}

extern "C" {

// ws: 6*W u64 (cnt[2W], start[2W], cursor[2W]); xchg: 3*W int64 (device)
// combined != 0: rec == blob == one buffer of per-destination [records | key
// bytes] segments (mr_pack_seg_bytes), sent with a single all-to-all.
int mr_pack_by_dest(const void* hi, const void* lo, const void* val, const void* rep, const void* part, u64 n, u32 W,
                    const void* src, void* ws, void* xchg, long long extra, void* rec, void* blob, int combined,
                    hipStream_t s) {
  if (W == 0 || W > (u32)pk::MAXW) return -1;
  unsigned long long* cnt = (unsigned long long*)ws;
  unsigned long long* start = cnt + 2 * W;
  unsigned long long* cursor = start + 2 * W;
  hipMemsetAsync(cnt, 0, 2 * W * sizeof(unsigned long long), s);
  if (n) {
    hipLaunchKernelGGL(pk::pk_count_kernel, dim3(pk_grid(n, 1024)), dim3(pk::T), 0, s, (const u64*)lo,
                       (const u64*)rep, (const u32*)part, n, W, cnt);
  }
  hipLaunchKernelGGL(pk::pk_scan_kernel, dim3(1), dim3(64), 0, s, (const unsigned long long*)cnt, W, start, cursor,
                     (long long*)xchg, extra, combined);
  if (n) {
    // one record per thread (the per-block reservation needs every key of the
    // block in flight at once): grid = ceil(n / 256), not capped
    const u64 g = (n + pk::T - 1) / pk::T;
    hipLaunchKernelGGL(pk::pk_scatter_kernel, dim3((unsigned)g), dim3(pk::T), 0, s, (const u64*)hi, (const u64*)lo,
                       (const long long*)val, (const u64*)rep, (const u32*)part, n, W, (const u8*)src,
                       (const unsigned long long*)start, cursor, (u8*)rec, (u8*)blob);
  }
  return (int)hipGetLastError();
}

// The send side from the map's table in three launches (cp_* above): ws =
// u64 [2W][nb] block counts (nb = ceil(cap / 512)) + 2W u64; buf (buf_cap
// bytes) receives the per-destination segments [records | key bytes];
// xchg = the count-exchange row [W][3]; rows_out (u64, device) = the table's
// occupied slots.  extra gets STATUS_REDO when the table overflowed, a chunk
// error word is set or the segments do not fit buf.
u64 mr_compact_pack_ws_bytes(u64 cap, u32 W) {
  const u64 nb = (cap + pk::CP * pk::CP_PER - 1) / (pk::CP * pk::CP_PER);
  return ((nb * 2 * W * 8 + 255) & ~255ull) + 2 * (u64)W * 8;
}

int mr_compact_pack(void* tag, void* hi, void* lo, void* val, void* rep, void* ctrl, u64 cap, u32 nparts, u32 W,
                    const void* src, void* ws, void* buf, u64 buf_cap, void* xchg, long long extra, const void* errs,
                    u32 nerr, void* rows_out, hipStream_t s) {
  if (W == 0 || W > (u32)pk::MAXW || cap == 0) return -1;
  GTab g = gtab_make(tag, val, ctrl, cap, (const u8*)src);
  const u64 nb = (cap + pk::CP * pk::CP_PER - 1) / (pk::CP * pk::CP_PER);
  unsigned long long* bcnt = (unsigned long long*)ws;
  unsigned long long* coltot = (unsigned long long*)((u8*)ws + ((nb * 2 * W * 8 + 255) & ~255ull));
  hipLaunchKernelGGL(pk::cp_count_kernel, dim3((unsigned)nb), dim3(pk::CP), 0, s, g, cap, nparts, W, (const u8*)src,
                     bcnt);
  hipLaunchKernelGGL(pk::cp_scan_kernel, dim3(2 * W), dim3(pk::CS), 0, s, bcnt, nb, coltot);
  hipLaunchKernelGGL(pk::cp_scatter_kernel, dim3((unsigned)nb), dim3(pk::CP), 2 * W * sizeof(unsigned long long), s, g,
                     cap, nparts, W, (const u8*)src, (const unsigned long long*)bcnt, (const unsigned long long*)coltot, (u8*)buf,
                     buf_cap, (long long*)xchg, extra, (const u32*)ctrl + 1, (const int*)errs, nerr,
                     (unsigned long long*)rows_out);
  return (int)hipGetLastError();
}

// src: the received key bytes the rep words index (combined layout: `rec`
// itself; may be null = no long-key byte verification)
int mr_insert_received(const void* rec, u64 n, const void* recv, u32 W, void* tag, void* hi, void* lo, void* val,
                       void* rep, void* ctrl, u64 cap, int op, int combined, const void* src, hipStream_t s) {
  if (n == 0) return 0;
  if (W == 0 || W > (u32)pk::MAXW_RECV) return -1;
  GTab g = gtab_make(tag, val, ctrl, cap, (const u8*)(combined ? rec : src));
  hipLaunchKernelGGL(pk::pk_insert_received_kernel, dim3(pk_grid(n, 2048)), dim3(256),
                     3 * (W + 1) * sizeof(long long), s, (const u8*)rec, n, (const long long*)recv, W, g, op, combined);
  return (int)hipGetLastError();
}

int mr_fix_loc(void* rec, u64 n, const void* rstart, const void* bstart, u32 W, void* rep_out, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(pk::pk_fix_loc_kernel, dim3(pk_grid(n)), dim3(256), 0, s, (u64*)rec, n, (const long long*)rstart,
                     (const long long*)bstart, W, (u64*)rep_out);
  return (int)hipGetLastError();
}

}  // extern "C"
