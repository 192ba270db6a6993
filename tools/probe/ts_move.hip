// ts_move.hip — TeraSort data-movement probe (not part of the framework):
// how fast can 100-byte rows be permuted on MI355X?
//   copy      : sequential copy (roofline reference)
//   gather    : out[i] = in[perm[i]]   (random 100-B row reads, sequential writes; the framework's ts_gather)
//   scatter   : out[inv[i]] = in[i]    (sequential reads, random 100-B row writes)
//   gather_w  : gather with perm random only inside windows of `win` rows (what an MSD bucket pass leaves)
// Built by tools/ts_move_probe.py (hipcc -> tools/probe/libtsmove.so).
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int WORDS = 25;

__global__ void copy_kernel(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) out[i] = in[i];
}

__global__ void gather_kernel(const uint32_t* __restrict__ in, const uint32_t* __restrict__ perm, uint64_t n,
                              uint32_t* __restrict__ out) {
  const uint64_t nw = n * WORDS;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += stride) {
    const uint64_t r = w / WORDS;
    const uint32_t j = (uint32_t)(w - r * WORDS);
    out[w] = __builtin_nontemporal_load(in + (uint64_t)perm[r] * WORDS + j);
  }
}

__global__ void scatter_kernel(const uint32_t* __restrict__ in, const uint32_t* __restrict__ inv, uint64_t n,
                               uint32_t* __restrict__ out) {
  const uint64_t nw = n * WORDS;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += stride) {
    const uint64_t r = w / WORDS;
    const uint32_t j = (uint32_t)(w - r * WORDS);
    out[(uint64_t)inv[r] * WORDS + j] = __builtin_nontemporal_load(in + w);
  }
}

// MSD bucket pass (probe): rows read in order into LDS (a tile of TR rows),
// bucket = top `bbits` bits of the first key byte, per-tile bucket counts ->
// one atomicAdd per bucket on per-bucket cursors (regions of `bcap` rows per
// bucket), rows written out of LDS grouped by bucket (runs of consecutive
// rows per bucket).  Also writes the row's top-32-bit key next to it in a key
// array of the same layout.
constexpr int BT = 512;
constexpr int TR = 1024;  // rows per tile: 100 KiB of LDS
__global__ void __launch_bounds__(BT) bucket_kernel(const uint32_t* __restrict__ in, uint64_t n, int bbits,
                                                   uint64_t bcap, unsigned long long* __restrict__ cursor,
                                                   uint32_t* __restrict__ out, uint32_t* __restrict__ keys) {
  __shared__ uint32_t rows[TR * WORDS];
  __shared__ uint32_t cnt[256];
  __shared__ uint32_t pos[256];
  __shared__ unsigned long long gbase[256];
  __shared__ uint16_t order[TR];
  __shared__ uint8_t bk[TR];
  const int t = threadIdx.x;
  const int nb = 1 << bbits;
  const uint64_t r0 = (uint64_t)blockIdx.x * TR;
  if (r0 >= n) return;
  const int nr = (int)min((uint64_t)TR, n - r0);
  for (int b = t; b < nb; b += BT) cnt[b] = 0;
  const uint32_t* src = in + r0 * WORDS;
  for (int w = t; w < nr * WORDS; w += BT) rows[w] = __builtin_nontemporal_load(src + w);
  __syncthreads();
  for (int r = t; r < nr; r += BT) {
    const uint32_t b = (rows[r * WORDS] & 0xFFu) >> (8 - bbits);
    bk[r] = (uint8_t)b;
    atomicAdd(&cnt[b], 1u);
  }
  __syncthreads();
  if (t == 0) {
    uint32_t a = 0;
    for (int b = 0; b < nb; ++b) {
      pos[b] = a;
      a += cnt[b];
    }
  }
  __syncthreads();
  for (int b = t; b < nb; b += BT) gbase[b] = cnt[b] ? atomicAdd(&cursor[b], (unsigned long long)cnt[b]) : 0ull;
  __syncthreads();
  for (int r = t; r < nr; r += BT) {
    const uint32_t k = atomicAdd(&pos[bk[r]], 1u);  // order inside a bucket: arbitrary (the sort fixes it)
    order[k] = (uint16_t)r;
  }
  __syncthreads();
  // out row for sorted slot k: bucket bk[order[k]], index gbase + (k - start of its run)
  // recompute run starts: pos[b] now holds the run END; start = end - cnt
  for (int w = t; w < nr * WORDS; w += BT) {
    const int k = w / WORDS, j = w - k * WORDS;
    const int r = order[k];
    const uint32_t b = bk[r];
    const uint64_t di = (uint64_t)b * bcap + gbase[b] + (uint64_t)(k - (int)(pos[b] - cnt[b]));
    out[di * WORDS + j] = rows[r * WORDS + j];
    if (j == 0) keys[di] = __builtin_bswap32(rows[r * WORDS]);
  }
}

extern "C" {
int probe_bucket(const void* in, uint64_t n, int bbits, uint64_t bcap, void* cursor, void* out, void* keys,
                 hipStream_t s) {
  hipLaunchKernelGGL(bucket_kernel, dim3((unsigned)((n + TR - 1) / TR)), dim3(BT), 0, s, (const uint32_t*)in, n,
                     bbits, bcap, (unsigned long long*)cursor, (uint32_t*)out, (uint32_t*)keys);
  return (int)hipGetLastError();
}
int probe_copy(const void* in, void* out, uint64_t nbytes, hipStream_t s) {
  hipLaunchKernelGGL(copy_kernel, dim3(16384), dim3(256), 0, s, (const uint4*)in, (uint4*)out, nbytes / 16);
  return (int)hipGetLastError();
}
int probe_gather(const void* in, const void* perm, uint64_t n, void* out, hipStream_t s) {
  hipLaunchKernelGGL(gather_kernel, dim3(16384), dim3(256), 0, s, (const uint32_t*)in, (const uint32_t*)perm, n,
                     (uint32_t*)out);
  return (int)hipGetLastError();
}
int probe_scatter(const void* in, const void* inv, uint64_t n, void* out, hipStream_t s) {
  hipLaunchKernelGGL(scatter_kernel, dim3(16384), dim3(256), 0, s, (const uint32_t*)in, (const uint32_t*)inv, n,
                     (uint32_t*)out);
  return (int)hipGetLastError();
}
}
