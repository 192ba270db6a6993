// Speculative home-slot probe: the (tag, lo, hi) words of a key's home slot,
// loaded together so several keys' probes are in flight at once.  home_hit:
// the key is at its home slot — a short key by its exact tag, a longer packed
// key by tag, lo and hi (slots are claimed once and hi is published before lo,
// so a matching triple is final); long keys (byte-verified) never hit here.
// A miss takes the full gtab_insert.
__device__ __forceinline__ void home_load(const GTab& g, u64 hi, u64 lo, u64& home, u64& st, u64& sl, u64& sh) {
  home = gtab_home(gtab_tag(hi, lo), g.mask);
  st = ld_agent(&g.tag[home]);
  sl = ld_agent(&g.lo[home]);
  sh = ld_agent(&g.hi[home]);
}

__device__ __forceinline__ bool home_hit(u64 hi, u64 lo, u64 st, u64 sl, u64 sh) {
  const u64 tag = gtab_tag(hi, lo);
  if (st != tag) return false;
  if (gtab_tag_exact(tag)) return true;
  return !key_is_long(lo) && sl == lo && sh == hi;
}

// Flush of an LDS combine table: each thread's claimed slots probe their home
// slots together, then fold there (hit) or through gtab_insert (miss).
// (spec = 0: no probes, every slot through gtab_insert — the A/B form)
__device__ __forceinline__ u32 cb_flush(const GTab& g, const Cols& c, const u64* tag, const u64* khi, const u64* klo,
                                        const u64* krep, const long long* acc, int spec) {
  constexpr int FL = CB_SLOTS / CB_T;
  const int t = threadIdx.x;
  u64 hm[FL], st[FL], sl[FL], sh[FL];
#pragma unroll
  for (int f = 0; f < FL; ++f) {
    const int s = t + f * CB_T;
    hm[f] = st[f] = sl[f] = sh[f] = 0;
    if (spec && tag[s]) home_load(g, khi[s], klo[s], hm[f], st[f], sl[f], sh[f]);
  }
  u32 claims = 0;
#pragma unroll
  for (int f = 0; f < FL; ++f) {
    const int s = t + f * CB_T;
    if (!tag[s]) continue;
    u64 slot = 0;
    int r = 1;
    if (spec && home_hit(khi[s], klo[s], st[f], sl[f], sh[f])) {
      slot = hm[f];
    } else {
      r = gtab_insert(g, khi[s], klo[s], 0, krep[s], OP_NONE, &slot);
      claims += r == 2;
    }
    if (r)
      for (int j = 0; j < c.k; ++j) cb_global_fold(c, j, slot, acc[j * CB_SLOTS + s]);
  }
  return claims;
}

