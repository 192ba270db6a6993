template <int C>
static void launch_gather_glds(const void* in, u64 nin, const void* perm, u64 n, int rb, void* out, hipStream_t s) {
  constexpr int R = C <= 8 ? 128 : 64;  // two images of R * C * 16 bytes
  const u64 nb = (n + R - 1) / R;
  const unsigned g = (unsigned)(nb < 65536 ? nb : 65536);
  hipLaunchKernelGGL((rc::rec_gather_glds_kernel<C, R>), dim3(g), dim3(256), 0, s, (const u8*)in, nin,
                     (const u32*)perm, n, (u32)rb, (u8*)out);
}

