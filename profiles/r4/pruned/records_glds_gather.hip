// The same gather with the row chunks moved global -> LDS by LDS-DMA loads
// (global_load_lds_dwordx4: no VGPR staging, the destination is the wave's
// 1 KiB slice of the image, lane-linear) into two images: batch b+1's loads
// are in flight while batch b's rows are stored from the other image, and the
// barrier after the stores drains them.  Needs in_bytes % 16 == 0 (every
// chunk is a whole 16-byte load); R * C is a multiple of 64, so a wave's
// slice never runs past an image.
// One LDS-DMA load of 16 bytes per lane into the wave's slice at LDS byte
// address lds_dst (wave-uniform), written as asm so the compiler's wait
// bookkeeping does not drain it at every later plain load or LDS read: the
// kernel counts it itself (s_waitcnt vmcnt(0) before the barrier that
// publishes the image).  M0 is set and restored in the same statement.
__device__ __forceinline__ void rc_glds16(const void* gsrc, u32 lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}

template <int C, int R>
__global__ void __launch_bounds__(256) rec_gather_glds_kernel(const u8* __restrict__ in, u64 nin,
                                                             const u32* __restrict__ perm, u64 n, u32 rb,
                                                             u8* __restrict__ out) {
  typedef u32 v4u __attribute__((ext_vector_type(4)));
  static_assert((R * C) % 64 == 0, "image slices of whole waves");
  __shared__ __attribute__((aligned(16))) v4u img0[R * C];
  __shared__ __attribute__((aligned(16))) v4u img1[R * C];
  __shared__ u32 mis0[R], mis1[R];
  constexpr int PER = (R * C + 255) / 256;
  const u32 t = threadIdx.x;
  const u32 wbase = t & ~63u;
  const u64 nbatch = (n + R - 1) / R;
  const u64 in_bytes = nin * (u64)rb;
  const float inv_rb = 1.0f / (float)rb;
  auto issue = [&](u64 bb, v4u* img, u32* mis) {
    const u64 q0 = bb * (u64)R;
    const u32 qrows = (u32)min((u64)R, n - q0);
    // every permutation entry first, then every chunk address (the waits for
    // those plain loads all happen here), then the LDS-DMA loads back to
    // back: any vmcnt wait after a DMA load would drain it too
    u32 pr[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const u32 idx = 256u * k + wbase + (t & 63u);
      const u32 row = idx / C;
      pr[k] = (idx < (u32)(R * C) && row < qrows) ? perm[q0 + row] : 0xFFFFFFFFu;
    }
    u64 a[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const u32 idx = 256u * k + wbase + (t & 63u);
      const u32 row = idx / C, c = idx - row * C;
      a[k] = 0;  // rows past the batch load chunk 0 of the input (never read)
      if (pr[k] != 0xFFFFFFFFu) {
        const u64 sb = (u64)clamp_row(pr[k], nin) * rb;
        a[k] = (sb & ~15ull) + 16ull * c;
        // a chunk past the input's end lies past this row's bytes (the input
        // ends on a 16-byte boundary): load a harmless one instead
        if (a[k] + 16 > in_bytes) a[k] = 0;
        if (c == 0) mis[row] = (u32)(sb & 15);
      }
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const u32 base = 256u * k + wbase;  // this wave's slice (wave-uniform)
      if (base >= (u32)(R * C)) continue;
      const u32 dst = __builtin_amdgcn_readfirstlane((u32)(uintptr_t)(&img[base]));
      rc_glds16(in + a[k], dst);
    }
  };
  auto store = [&](u64 bb, const v4u* img, const u32* mis) {
    const u64 r0 = bb * (u64)R;
    const u32 rows = (u32)min((u64)R, n - r0);
    const u32* img32 = reinterpret_cast<const u32*>(img);
    const u32 obytes = rows * rb;
    u8* ob = out + r0 * rb;
    const u32 nch = obytes >> 4;
    for (u32 oc = t; oc < nch + 1; oc += 256) {
      const u32 byte0 = oc * 16u;
      if (byte0 >= obytes) break;
      u32 row = (u32)((float)byte0 * inv_rb);
      if (row * rb > byte0) --row;
      if ((row + 1) * rb <= byte0) ++row;
      const u32 off = byte0 - row * rb;
      u32 w[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        u32 rr = row, oo = off + 4u * j;
        if (oo >= rb) {
          ++rr;
          oo -= rb;
        }
        w[j] = rr < rows ? img32[(rr * (u32)C * 16u + mis[rr] + oo) >> 2] : 0u;
      }
      if (oc < nch) {
        __builtin_nontemporal_store(v4u{w[0], w[1], w[2], w[3]}, reinterpret_cast<v4u*>(ob + byte0));
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (byte0 + 4u * j < obytes) *reinterpret_cast<u32*>(ob + byte0 + 4u * j) = w[j];
      }
    }
  };
  u64 b = blockIdx.x;
  if (b < nbatch) issue(b, img0, mis0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the DMA loads are not in the compiler's count)
  __syncthreads();
  while (b < nbatch) {
    const u64 b1 = b + gridDim.x;
    if (b1 < nbatch) issue(b1, img1, mis1);
    store(b, img0, mis0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (b1 >= nbatch) break;
    const u64 b2 = b1 + gridDim.x;
    if (b2 < nbatch) issue(b2, img0, mis0);
    store(b1, img1, mis1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    b = b2;
  }
}

