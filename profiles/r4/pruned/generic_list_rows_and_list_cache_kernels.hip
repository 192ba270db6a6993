// List mode, one row per thread-item (LR_ITEMS rows per thread, strided by the
// block): the rows' span and key loads are issued together, then every row's
// home-slot probe (home_load); a row whose key sits at its home slot (a
// sparse table: most rows) takes that slot with no further memory round trip,
// the others the full insert.  Each row then writes its
// posting (slot, value) at its row index.
constexpr int LR_T = 256, LR_ITEMS = 6;
__global__ void __launch_bounds__(LR_T) list_rows_kernel(GTab g, Keys ks, u64 n, Cols c) {
  const int t = threadIdx.x;
  u32 claims = 0;
  for (u64 r0 = (u64)blockIdx.x * (LR_T * LR_ITEMS); r0 < n; r0 += (u64)gridDim.x * (LR_T * LR_ITEMS)) {
    u64 khi_r[LR_ITEMS], klo_r[LR_ITEMS], krep_r[LR_ITEMS];
    const u32 ok = cb_row_keys<LR_ITEMS, LR_T>(ks, r0, LR_ITEMS, n, khi_r, klo_r, krep_r);
    u64 home[LR_ITEMS], st[LR_ITEMS], sl[LR_ITEMS], sh[LR_ITEMS];
#pragma unroll
    for (int it = 0; it < LR_ITEMS; ++it) {
      home[it] = st[it] = sl[it] = sh[it] = 0;
      if (ok & (1u << it)) home_load(g, khi_r[it], klo_r[it], home[it], st[it], sl[it], sh[it]);
    }
#pragma unroll
    for (int it = 0; it < LR_ITEMS; ++it) {
      const u64 i = r0 + (u64)it * LR_T + t;
      if (i >= n) continue;
      long long slot = -1;
      if (ok & (1u << it)) {
        if (home_hit(khi_r[it], klo_r[it], st[it], sl[it], sh[it])) {
          slot = (long long)home[it];
        } else {
          u64 sl = 0;
          const int r = gtab_insert(g, khi_r[it], klo_r[it], 0, krep_r[it], OP_NONE, &sl);
          claims += r == 2;
          slot = r ? (long long)sl : -1ll;
        }
      }
      c.post_slot[c.post_base + i] = slot;
      ((long long*)c.dst[0])[c.post_base + i] =
          c.dtype[0] == VT_F64 ? __double_as_longlong(rd_f64(c, 0, i)) : rd_i64(c, 0, i);
    }
  }
  gtab_count_claims(g, claims);
}

// List mode (postings: one (slot, value) per row, in row order), rows of a
// block resolved through an LDS key -> global-slot cache: the block's rows
// claim LDS slots (cb_slot), each distinct key of the block is inserted into
// the HBM table ONCE, and every row then writes its posting with its key's
// slot — a Zipf vocabulary's hot keys no longer probe the HBM table per row
// (agg_insert_kernel did).  Keys the cache cannot hold (full, long keys) take
// the direct insert.
__global__ void __launch_bounds__(CB_T) list_combine_kernel(GTab g, Keys ks, u64 n, Cols c, u32 rows) {
  constexpr int CB_ITEMS = CB_ROWS / CB_T;
  const int items = (int)(rows / CB_T);
  extern __shared__ __attribute__((aligned(16))) u64 lds[];
  u64* tag = lds;
  u64* khi = tag + CB_SLOTS;
  u64* klo = khi + CB_SLOTS;
  u64* krep = klo + CB_SLOTS;
  long long* gslot = (long long*)(krep + CB_SLOTS);  // global slot of each cached key (-1: overflow)
  __shared__ u32 nclaimed;
  const int t = threadIdx.x;
  for (int s = t; s < CB_SLOTS; s += CB_T) {
    tag[s] = 0;
    klo[s] = 0;
  }
  if (t == 0) nclaimed = 0;
  __syncthreads();
  u32 claims = 0;
  const u64 r0 = (u64)blockIdx.x * rows;
  u64 khi_r[CB_ITEMS], klo_r[CB_ITEMS], krep_r[CB_ITEMS];
  const u32 ok = cb_row_keys<CB_ITEMS>(ks, r0, items, n, khi_r, klo_r, krep_r);
  int s_r[CB_ITEMS];
#pragma unroll
  for (int it = 0; it < CB_ITEMS; ++it) {
    s_r[it] = -1;
    if (ok & (1u << it))
      s_r[it] = key_is_long(klo_r[it]) ? -1 : cb_slot(tag, khi, klo, krep, &nclaimed, khi_r[it], klo_r[it], krep_r[it]);
  }
  __syncthreads();
  for (int s = t; s < CB_SLOTS; s += CB_T) {
    if (!tag[s]) continue;
    u64 slot = 0;
    const int r = gtab_insert(g, khi[s], klo[s], 0, krep[s], OP_NONE, &slot);
    claims += r == 2;
    gslot[s] = r ? (long long)slot : -1ll;
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < CB_ITEMS; ++it) {
    const u64 i = r0 + (u64)it * CB_T + t;
    if (it >= items || i >= n) continue;
    long long slot = -1;
    if (s_r[it] >= 0) {
      slot = gslot[s_r[it]];
    } else if (ok & (1u << it)) {
      u64 sl = 0;
      const int r = gtab_insert(g, khi_r[it], klo_r[it], 0, krep_r[it], OP_NONE, &sl);
      claims += r == 2;
      slot = r ? (long long)sl : -1ll;
    }
    c.post_slot[c.post_base + i] = slot;
    ((long long*)c.dst[0])[c.post_base + i] =
        c.dtype[0] == VT_F64 ? __double_as_longlong(rd_f64(c, 0, i)) : rd_i64(c, 0, i);
  }
  gtab_count_claims(g, claims);
}

