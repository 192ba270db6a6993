// sort11.hip — onesweep LSD radix passes over u32 keys with 11-bit digits
// (2048 bins): 32-bit key prefixes in THREE passes (11 + 11 + 10 bits)
// instead of four 8-bit ones (sort.hip), for the record plane's TeraSort sort
// of 100 M 32-bit prefixes ("11-bit digits, 3 passes").
//
// Same structure as sort.hip's rs_onesweep_kernel: tiles taken in dispatch
// order, wave-private ballot ranking (11 ballots per round instead of 8),
// LDS image of the tile in digit order, decoupled look-back on tagged 64-bit
// granules — but every thread owns 8 consecutive bins (2048 / 256) for the
// tile histogram, the scans and the look-back, and a tile publishes 2048
// granules.  The trade: one pass less over the keys and values (8 bytes read
// + 8 written per key and pass) against 8x the look-back granules per tile and
// shorter digit runs in the scattered writes (2048 bins over a tile).
#include <hip/hip_runtime.h>
#include "mr_common.h"

namespace mr {
namespace r11 {

constexpr int T = 256;
constexpr int WAVES = T / 64;
constexpr int BINS = 2048;
constexpr int BPT = BINS / T;  // bins per thread
// LDS bin arrays are padded by one word per 8 bins: thread t's bins t*8..t*8+7
// sit at t*9..t*9+7, so the 64 lanes of a wave walking "their j-th bin" hit 64
// different banks (unpadded, a stride of 8 words: 8 lanes per bank, 8-way
// conflicts on every per-thread histogram, scan and offset access)
constexpr int PBINS = BINS + BINS / BPT;
static_assert(BPT == 8, "pb() pads one word per 8 bins");
__device__ __forceinline__ u32 pb(u32 b) { return b + (b >> 3); }
constexpr u64 GR_AGG = 1ull, GR_INC = 2ull;

__device__ __forceinline__ u64 gr_pack(u32 epoch, u64 flag, u64 count) {
  return ((u64)(epoch & 0xFFFFFFu) << 40) | (flag << 38) | (count & ((1ull << 38) - 1));
}

__device__ __forceinline__ u32 block_scan(u32 v, u32* tmp) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const u32 y = __shfl_up(v, o);
    if (lane >= o) v += y;
  }
  __syncthreads();
  if (lane == 63) tmp[wave] = v;
  __syncthreads();
  u32 add = 0;
#pragma unroll
  for (int w = 0; w < WAVES; ++w) add += w < wave ? tmp[w] : 0u;
  return v + add;
}

// The 3 digit histograms ([3][2048]: bits 0-10, 11-21, 22-31) of u32 keys.
__global__ void __launch_bounds__(T) hist11_kernel(const u32* __restrict__ keys, u64 n, u32* __restrict__ ghist) {
  __shared__ u32 h[3][BINS];
  const int t = threadIdx.x;
  for (int i = t; i < 3 * BINS; i += T) (&h[0][0])[i] = 0;
  __syncthreads();
  const u64 stride = (u64)gridDim.x * T;
  for (u64 i = (u64)blockIdx.x * T + t; i < n; i += stride) {
    const u32 k = keys[i];
    atomicAdd(&h[0][k & 0x7FF], 1u);
    atomicAdd(&h[1][(k >> 11) & 0x7FF], 1u);
    atomicAdd(&h[2][k >> 22], 1u);
  }
  __syncthreads();
  for (int i = t; i < 3 * BINS; i += T)
    if ((&h[0][0])[i]) atomicAdd(&ghist[i], (&h[0][0])[i]);
}

template <int ROUNDS>
__global__ void __launch_bounds__(T) onesweep11_kernel(const u32* keys_in, const u32* vals_in, u32* keys_out,
                                                       u32* vals_out, u64 n, int shift, u32 mask, const u32* ghist,
                                                       u64* granules, u32* tile_counter, u32 epoch, u32* err, int iota) {
  constexpr int TILE = T * ROUNDS;
  constexpr int SUB = TILE / WAVES;
  __shared__ u32 sk[TILE];
  __shared__ u32 sv[TILE];
  __shared__ u32 wc[WAVES][PBINS];
  __shared__ u32 gout[PBINS];
  __shared__ u32 wsum[WAVES];
  __shared__ u32 sh_tile;
  __shared__ u32 sh_uniform;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  if (t == 0) {
    sh_tile = atomicAdd(tile_counter, 1u);
    sh_uniform = 0;
  }
  for (int i = t; i < WAVES * PBINS; i += T) (&wc[0][0])[i] = 0;
  u32 gcnt[BPT];
  u32 gsum = 0;
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    gcnt[j] = ghist[t * BPT + j];
    gsum += gcnt[j];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < BPT; ++j)
    if (gcnt[j] == n) sh_uniform = 1;
  const u32 gex = block_scan(gsum, wsum) - gsum;  // (its barriers also publish sh_uniform)
  __syncthreads();
  const u32 tile = sh_tile;
  const u64 t0 = (u64)tile * TILE;
  if (sh_uniform) {  // every key has this digit: order unchanged
    for (int r = 0; r < ROUNDS; ++r) {
      const u64 i = t0 + (u64)r * T + t;
      if (i < n) {
        keys_out[i] = keys_in[i];
        vals_out[i] = vals_in ? vals_in[i] : (u32)i;
      }
    }
    return;
  }
  const u64 w0 = t0 + (u64)wave * SUB;
  u32 kr[ROUNDS], vr[ROUNDS], myrank[ROUNDS];
#pragma unroll
  for (int r = 0; r < ROUNDS; ++r) {
    const u64 i = w0 + (u64)r * 64 + lane;
    kr[r] = i < n ? keys_in[i] : 0u;
    vr[r] = (i < n && vals_in) ? vals_in[i] : (iota ? (u32)i : 0u);
  }
  const unsigned long long below = (1ull << lane) - 1ull;
  u32* mywc = wc[wave];
#pragma unroll
  for (int r = 0; r < ROUNDS; ++r) {
    const u64 i = w0 + (u64)r * 64 + lane;
    const bool valid = i < n;
    const u32 d = (kr[r] >> shift) & mask;
    unsigned long long peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 11; ++b) {
      const unsigned long long m = __ballot((d >> b) & 1u);
      peers &= ((d >> b) & 1u) ? m : ~m;
    }
    const u32 before = valid ? mywc[pb(d)] : 0u;
    myrank[r] = before + (u32)__popcll(peers & below);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): every lane read its counter before the leader updates it
    if (valid && (peers & below) == 0) mywc[pb(d)] = before + (u32)__popcll(peers);
  }
  __syncthreads();
  u32 mine[BPT];
  u32 msum = 0;
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    const int b = t * (BPT + 1) + j;  // pb(t * BPT + j)
    u32 c = 0;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) c += wc[w][b];
    mine[j] = c;
    msum += c;
  }
  u64* G = granules + (u64)tile * BINS + (u64)t * BPT;
#pragma unroll
  for (int j = 0; j < BPT; ++j)
    __hip_atomic_store(&G[j], gr_pack(epoch, tile == 0 ? GR_INC : GR_AGG, mine[j]), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  const u32 lex = block_scan(msum, wsum) - msum;
  u32 lbase[BPT], gbase[BPT];
  {
    u32 off = lex, goff = gex;
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      const int b = t * (BPT + 1) + j;  // pb(t * BPT + j)
      lbase[j] = off;
      gbase[j] = goff;
      u32 o = off;
#pragma unroll
      for (int w = 0; w < WAVES; ++w) {
        const u32 c = wc[w][b];
        wc[w][b] = o;  // now: LDS start of wave w's keys of digit b
        o += c;
      }
      off += mine[j];
      goff += gcnt[j];
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < ROUNDS; ++r) {
    const u64 i = w0 + (u64)r * 64 + lane;
    if (i < n) {
      const u32 d = (kr[r] >> shift) & mask;
      const u32 pos = mywc[pb(d)] + myrank[r];
      sk[pos] = kr[r];
      sv[pos] = vr[r];
    }
  }
  // decoupled look-back of this thread's 8 bins, all walked together
  u64 excl[BPT];
#pragma unroll
  for (int j = 0; j < BPT; ++j) excl[j] = 0;
  if (tile > 0) {
    long long jt[BPT];
#pragma unroll
    for (int j = 0; j < BPT; ++j) jt[j] = (long long)tile - 1;
    u32 done = 0, spins = 0;
    while (done != (1u << BPT) - 1u) {
      bool waiting = false;
#pragma unroll
      for (int j = 0; j < BPT; ++j) {
        if (done & (1u << j)) continue;
        const u64 g = __hip_atomic_load(&granules[(u64)jt[j] * BINS + (u64)t * BPT + j], __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
        const u64 fl = (g >> 38) & 3ull;
        if ((u32)(g >> 40) != (epoch & 0xFFFFFFu) || fl == 0) {
          waiting = true;
          continue;
        }
        excl[j] += g & ((1ull << 38) - 1);
        if (fl == GR_INC) done |= 1u << j;
        else --jt[j];
      }
      if (waiting) {
        if (++spins > (1u << 22)) {
          atomicOr(err, 1u);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
#pragma unroll
    for (int j = 0; j < BPT; ++j)
      __hip_atomic_store(&G[j], gr_pack(epoch, GR_INC, excl[j] + mine[j]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#pragma unroll
  for (int j = 0; j < BPT; ++j) gout[t * (BPT + 1) + j] = gbase[j] + (u32)excl[j] - lbase[j];
  __syncthreads();
  const u32 cnt = (u32)min((u64)TILE, n - t0);
  for (u32 i = t; i < cnt; i += T) {
    const u32 k = sk[i];
    const u32 pos = gout[pb((k >> shift) & mask)] + i;
    keys_out[pos] = k;
    vals_out[pos] = sv[i];
  }
}

}  // namespace r11
}  // namespace mr

using namespace mr;

static int g_r11_rounds = 16;

extern "C" {

// keys per thread of the 11-bit tiles (16: two workgroups per CU; 24 / 32: one)
int mr_sort11_set_rounds(int rounds) {
  if (rounds != 8 && rounds != 16 && rounds != 24 && rounds != 32) return -1;
  g_r11_rounds = rounds;
  return 0;
}

u64 mr_sort11_tiles(u64 n) {
  const u64 tile = (u64)r11::T * (u64)g_r11_rounds;
  return (n + tile - 1) / tile;
}

// ghist: zeroed u32 [3][2048]
int mr_hist11(const void* keys, u64 n, void* ghist, hipStream_t s) {
  if (n == 0) return 0;
  u64 g = (n + 4 * r11::T - 1) / (4 * r11::T);
  if (g > 1024) g = 1024;
  hipLaunchKernelGGL(r11::hist11_kernel, dim3((unsigned)g), dim3(r11::T), 0, s, (const u32*)keys, n, (u32*)ghist);
  return (int)hipGetLastError();
}

// One 11-bit pass: digit (key >> shift) & mask (mask 0x7FF, or 0x3FF for the
// top 10 bits); ghist = that digit's 2048-bin histogram; granules: u64
// [mr_sort11_tiles(n)][2048]; tile_counter zeroed; vals_in null + iota: the
// value of key i is i.
int mr_radix_onesweep11(const void* keys_in, const void* vals_in, void* keys_out, void* vals_out, u64 n, int shift,
                        u32 mask, const void* ghist, void* granules, void* tile_counter, u32 epoch, void* err, int iota,
                        hipStream_t s) {
  if (n == 0) return 0;
  const u32 nt = (u32)mr_sort11_tiles(n);
#define R11_LAUNCH(R)                                                                                               \
  hipLaunchKernelGGL((r11::onesweep11_kernel<R>), dim3(nt), dim3(r11::T), 0, s, (const u32*)keys_in,               \
                     (const u32*)vals_in, (u32*)keys_out, (u32*)vals_out, n, shift, mask, (const u32*)ghist,        \
                     (u64*)granules, (u32*)tile_counter, epoch, (u32*)err, iota)
  switch (g_r11_rounds) {
    case 8: R11_LAUNCH(8); break;
    case 24: R11_LAUNCH(24); break;
    case 32: R11_LAUNCH(32); break;
    default: R11_LAUNCH(16);
  }
#undef R11_LAUNCH
  return (int)hipGetLastError();
}

}  // extern "C"
