// Probe: random-address 64-bit atomic add / CAS throughput into an HBM table,
// agent scope vs workgroup scope (is a workgroup-scope global atomic executed
// in the XCD's L2?), plus the XCC_ID hardware register distribution.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33; return x;
}

template <int SCOPE, int KIND>
__global__ void __launch_bounds__(256) probe(unsigned long long* tab, uint64_t mask, int iters, uint64_t salt) {
  uint64_t s = mix((uint64_t)blockIdx.x * 256 + threadIdx.x + salt);
  for (int i = 0; i < iters; ++i) {
    s = mix(s + i);
    unsigned long long* p = tab + (s & mask);
    if (KIND == 0) {
      __hip_atomic_fetch_add(p, 1ull, __ATOMIC_RELAXED, SCOPE);
    } else if (KIND == 1) {
      unsigned long long e = 0;
      __hip_atomic_compare_exchange_strong(p, &e, s | 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED, SCOPE);
    } else if (KIND == 3) {
      // hot addresses: every workgroup adds to the same `mask+1` words, 8 B
      // apart (one per lane group) -- contention of a popular key's counter
      __hip_atomic_fetch_add(tab + ((threadIdx.x + i) & mask) * 16, 1ull, __ATOMIC_RELAXED, SCOPE);
    } else {
      unsigned long long v = __hip_atomic_fetch_add(p, 1ull, __ATOMIC_RELAXED, SCOPE);
      if (v == 0xFFFFFFFFFFFFull) tab[0] = v;
    }
  }
}

__global__ void xcc(unsigned* out) {
  if (threadIdx.x == 0) {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    out[blockIdx.x] = v;
  }
}

template <int SCOPE, int KIND>
float run(unsigned long long* tab, uint64_t mask, int blocks, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  probe<SCOPE, KIND><<<blocks, 256>>>(tab, mask, iters, 1);
  hipEventRecord(a);
  probe<SCOPE, KIND><<<blocks, 256>>>(tab, mask, iters, 2);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  const uint64_t n = 1ull << 22;  // 32 MiB of u64
  unsigned long long* tab;
  hipMalloc(&tab, n * 8);
  hipMemset(tab, 0, n * 8);
  const int blocks = 4096, iters = 64;
  const double ops = (double)blocks * 256 * iters;
  struct { const char* name; float ms; } r[] = {
    {"add  agent    ", run<__HIP_MEMORY_SCOPE_AGENT, 0>(tab, n - 1, blocks, iters)},
    {"add  workgroup", run<__HIP_MEMORY_SCOPE_WORKGROUP, 0>(tab, n - 1, blocks, iters)},
    {"cas  agent    ", run<__HIP_MEMORY_SCOPE_AGENT, 1>(tab, n - 1, blocks, iters)},
    {"cas  workgroup", run<__HIP_MEMORY_SCOPE_WORKGROUP, 1>(tab, n - 1, blocks, iters)},
    {"addr agent    ", run<__HIP_MEMORY_SCOPE_AGENT, 2>(tab, n - 1, blocks, iters)},
    {"addr workgroup", run<__HIP_MEMORY_SCOPE_WORKGROUP, 2>(tab, n - 1, blocks, iters)},
    {"add  agent 1MiB", run<__HIP_MEMORY_SCOPE_AGENT, 0>(tab, (1 << 17) - 1, blocks, iters)},
    {"hot 1 addr     ", run<__HIP_MEMORY_SCOPE_AGENT, 3>(tab, 0, 64, iters)},
    {"hot 16 addr    ", run<__HIP_MEMORY_SCOPE_AGENT, 3>(tab, 15, 64, iters)},
    {"hot 256 addr   ", run<__HIP_MEMORY_SCOPE_AGENT, 3>(tab, 255, 64, iters)},
    {"hot 4096 addr  ", run<__HIP_MEMORY_SCOPE_AGENT, 3>(tab, 4095, 64, iters)},
    {"add  wg    1MiB", run<__HIP_MEMORY_SCOPE_WORKGROUP, 0>(tab, (1 << 17) - 1, blocks, iters)},
  };
  int i = 0;
  for (auto& x : r) {
    const double o = (i++ >= 8) ? 64.0 * 256 * iters : ops;
    printf("%s %8.3f ms  %7.2f G atomics/s\n", x.name, x.ms, o / x.ms / 1e6);
  }
  unsigned* d; hipMalloc(&d, 4096 * 4);
  xcc<<<4096, 64>>>(d);
  std::vector<unsigned> h(4096);
  hipMemcpy(h.data(), d, 4096 * 4, hipMemcpyDeviceToHost);
  int hist[32] = {0}; int bad = 0, rr = 0;
  for (int i = 0; i < 4096; ++i) { if (h[i] < 32) hist[h[i]]++; else bad++; if (h[i] % 16 == (unsigned)(i % 8)) rr++; }
  printf("xcc_id histogram:"); for (int i = 0; i < 16; ++i) printf(" %d", hist[i]); printf("  (>=32: %d)\n", bad);
  printf("first 16 ids:"); for (int i = 0; i < 16; ++i) printf(" %u", h[i]); printf("  blockIdx%%8==xcc: %d/4096\n", rr);
  return 0;
}
