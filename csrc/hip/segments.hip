// segments.hip — segmented folds over CSR value lists (the batched reducer
// plane of parallel/reducers.py and ops/segments.py).
//
// Reference semantics (/root/reference/mapreduce/job.lua:98-112,264-284): the
// reducer (and the combiner, the reduce module's ``combinerfn``, task.lua:325)
// folds each key's whole value list.  On the device a rank's keys and their
// lists are one CSR pair: off[m + 1] (int64) and val[n]; segment s = values
// val[off[s] .. off[s+1]).  Lists are heavily skewed — a hot key holds millions
// of values, most keys a handful — so the work is split by VALUES, not keys:
//
//   * a thread folds V consecutive values (a tile of 256 * V per workgroup);
//     a segment lying wholly inside one thread's range is stored directly;
//   * the partial folds of segments crossing thread boundaries (at most two
//     per thread: the head that started before the thread, the tail that goes
//     on after it) are combined across the 64-lane wavefront by a segmented
//     Hillis-Steele scan over __shfl_up (keys are non-decreasing along the
//     lanes, so equal keys at both ends of a lane span mean one run);
//   * one global atomic per (wavefront, crossing segment) merges wavefronts.
//
// A hot key of 3 M values thus takes ~3 M / (64 * V) atomics instead of one
// per value, and a tile of singletons takes none.  The segment of a thread's
// first value is found by binary search in off[], narrowed to the segments of
// the workgroup's tile (two searches per workgroup, in LDS broadcast).
//
// Empty segments keep the caller's fill (the fold's identity).
#include <hip/hip_runtime.h>
#include <climits>
#include "mr_common.h"

namespace mr {
namespace seg {

constexpr int THREADS = 256;
constexpr int V = 8;                      // values per thread
constexpr int TILE = THREADS * V;         // values per workgroup
enum Op : int { SUM = 0, MIN = 1, MAX = 2 };

template <typename T>
__device__ __forceinline__ T fold(T a, T b, int op) {
  if (op == MIN) return b < a ? b : a;
  if (op == MAX) return b > a ? b : a;
  return a + b;
}

template <typename T>
__device__ __forceinline__ void atomic_fold(T* p, T v, int op) {
  if (op == MIN) __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else if (op == MAX) __hip_atomic_fetch_max(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// largest s in [lo, hi] with off[s] <= i  (off non-decreasing; off[lo] <= i)
__device__ __forceinline__ long long seg_of(const long long* __restrict__ off, long long lo, long long hi,
                                            long long i) {
  while (lo < hi) {
    long long mid = (lo + hi + 1) >> 1;
    if (off[mid] <= i) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

template <typename T>
__device__ __forceinline__ T shfl_up_t(T v, int d) {
  if constexpr (sizeof(T) == 8) {
    long long b;
    __builtin_memcpy(&b, &v, 8);
    b = __shfl_up(b, d, 64);
    T r;
    __builtin_memcpy(&r, &b, 8);
    return r;
  } else {
    return __shfl_up(v, d, 64);
  }
}

template <typename T>
__global__ void __launch_bounds__(THREADS) seg_reduce_kernel(const long long* __restrict__ off, long long m,
                                                             const T* __restrict__ val, long long n, int op,
                                                             T* __restrict__ out) {
  __shared__ long long s_range[2];
  const long long tile0 = (long long)blockIdx.x * TILE;
  if (threadIdx.x == 0) {
    long long last = tile0 + TILE - 1 < n - 1 ? tile0 + TILE - 1 : n - 1;
    // off[0] == 0 <= tile0: the searches start from segment 0
    long long a = seg_of(off, 0, m - 1, tile0);
    long long b = seg_of(off, a, m - 1, last);
    s_range[0] = a;
    s_range[1] = b;
  }
  __syncthreads();
  const long long sa = s_range[0], sb = s_range[1];
  const long long t0 = tile0 + (long long)threadIdx.x * V;
  const long long t1 = t0 + V < n ? t0 + V : n;

  // head: partial fold of a segment that started before t0 and ends inside
  // [t0, t1); tail: partial fold of the segment that goes on past t1 (or
  // started before t0 and ends exactly at t1)
  long long hs = -1, ts = -1;
  T hv = T(0), tv = T(0);
  if (t0 < t1) {
    T x[V];
    if (t0 + V <= n) {
#pragma unroll
      for (int k = 0; k < V; ++k) x[k] = val[t0 + k];
    } else {
#pragma unroll
      for (int k = 0; k < V; ++k) x[k] = t0 + k < n ? val[t0 + k] : T(0);
    }
    long long s = seg_of(off, sa, sb, t0);
    long long end = off[s + 1];
    bool started_here = off[s] >= t0;
    T acc = x[0];
#pragma unroll
    for (int k = 1; k <= V; ++k) {
      const long long i = t0 + k;
      if (i > t1) break;
      if (i == end || i == t1) {
        // segment s's values in this thread end here
        if (started_here && i == end) {
          out[s] = acc;  // wholly inside this thread
        } else if (i == end) {
          hs = s;        // started before t0, ends here
          hv = acc;
        } else {
          ts = s;        // goes on past t1
          tv = acc;
        }
        if (i == t1) break;
        // next non-empty segment: the one holding value i
        s = off[s + 2] > i ? s + 1 : seg_of(off, s + 1, sb, i);
        end = off[s + 1];
        started_here = true;
        acc = x[k < V ? k : V - 1];
      } else {
        acc = fold(acc, x[k < V ? k : V - 1], op);
      }
    }
  }
  // segmented inclusive scan of the tails along the lanes
  const int lane = threadIdx.x & 63;
  T S = tv;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    long long k = __shfl_up(ts, d, 64);
    T o = shfl_up_t(S, d);
    if (lane >= d && ts >= 0 && k == ts) S = fold(S, o, op);
  }
  long long prev_key = __shfl_up(ts, 1, 64);
  T prev_S = shfl_up_t(S, 1);
  long long next_key = __shfl_down(ts, 1, 64);
  long long next_head = __shfl_down(hs, 1, 64);
  if (hs >= 0) {
    T v = hv;
    if (lane > 0 && prev_key == hs) v = fold(v, prev_S, op);
    atomic_fold(out + hs, v, op);
  }
  if (ts >= 0) {
    bool continues = lane < 63 && (next_key == ts || next_head == ts);
    if (!continues) atomic_fold(out + ts, S, op);
  }
}

// Key index of each posting: pos[pslot[i]] for a posting of a listed slot,
// `none` for a dropped row (pslot < 0) or a slot past the table, as u32 (one
// pass in place of torch's clamp + gather + where), plus the radix sort's
// digit histograms of those u32 keys ([8][256] layout, the first 4 rows;
// LDS-combined per block) so the stable u32 sort needs no histogram pass.
__global__ void __launch_bounds__(256) posting_keys_kernel(const long long* __restrict__ pos, long long space,
                                                          const long long* __restrict__ pslot, long long n,
                                                          unsigned none, unsigned* __restrict__ out,
                                                          unsigned* __restrict__ ghist) {
  __shared__ unsigned h[4][256];
  const int t = threadIdx.x;
#pragma unroll
  for (int b = 0; b < 4; ++b) h[b][t] = 0;
  __syncthreads();
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + t; i < n; i += stride) {
    const long long s = pslot[i];
    const unsigned k = (s >= 0 && s < space) ? (unsigned)pos[s] : none;
    out[i] = k;
#pragma unroll
    for (int b = 0; b < 4; ++b) atomicAdd(&h[b][(k >> (8 * b)) & 0xFFu], 1u);
  }
  __syncthreads();
#pragma unroll
  for (int b = 0; b < 4; ++b)
    if (h[b][t]) atomicAdd(&ghist[b * 256 + t], h[b][t]);
}

}  // namespace seg
}  // namespace mr

extern "C" {

// ghist: zeroed u32[8][256] (rows 0-3 are filled)
int mr_posting_keys(const void* pos, long long space, const void* pslot, long long n, long long none, void* out,
                    void* ghist, hipStream_t stream) {
  using namespace mr::seg;
  if (n <= 0) return 0;
  if (none < 0 || none > 0xFFFFFFFFll || !ghist) return -1;
  long long g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(posting_keys_kernel, dim3((unsigned)g), dim3(256), 0, stream, (const long long*)pos, space,
                     (const long long*)pslot, n, (unsigned)none, (unsigned*)out, (unsigned*)ghist);
  return (int)hipGetLastError();
}

// out[s] = fold of val[off[s] .. off[s+1]) for s < m (out pre-filled with the
// fold's identity by the caller; empty segments keep it).  vtype: 0 int64,
// 1 float64; op: 0 sum, 1 min, 2 max.  off: int64[m + 1], off[0] == 0,
// off[m] == n, non-decreasing.
int mr_seg_reduce(const void* off, unsigned long long m, const void* val, unsigned long long n, int vtype, int op,
                  void* out, hipStream_t stream) {
  using namespace mr::seg;
  if (n == 0 || m == 0) return 0;
  if (op < 0 || op > 2 || vtype < 0 || vtype > 1) return -1;
  unsigned long long blocks = (n + TILE - 1) / TILE;
  if (vtype == 0)
    hipLaunchKernelGGL(seg_reduce_kernel<long long>, dim3((unsigned)blocks), dim3(THREADS), 0, stream,
                       (const long long*)off, (long long)m, (const long long*)val, (long long)n, op, (long long*)out);
  else
    hipLaunchKernelGGL(seg_reduce_kernel<double>, dim3((unsigned)blocks), dim3(THREADS), 0, stream,
                       (const long long*)off, (long long)m, (const double*)val, (long long)n, op, (double*)out);
  return (int)hipGetLastError();
}

}  // extern "C"
