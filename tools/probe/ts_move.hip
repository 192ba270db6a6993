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

extern "C" {
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
