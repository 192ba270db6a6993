  if (a->list && a->rows_only == 1) {  // (2: the one-row-per-thread kernel below, for A/B)
    u64 g = (n + LR_T * LR_ITEMS - 1) / (LR_T * LR_ITEMS);
    if (g > 16384) g = 16384;
    hipLaunchKernelGGL(list_rows_kernel, dim3((unsigned)g), dim3(LR_T), 0, stream,
                       ag_gtab(tag, thi, tlo, tval, trep, ctrl, cap, src), ks, n, to_cols(a));
    return (int)hipGetLastError();
  }
  if (a->list && !a->rows_only && n >= (u64)CB_ROWS) {
    const size_t lds = (size_t)CB_SLOTS * 5 * sizeof(u64);
    u32 rows = (u32)CB_ROWS;
    while (rows > (u32)CB_T && (n + rows - 1) / rows < 1024) rows >>= 1;
    const u64 nb = (n + rows - 1) / rows;
    hipLaunchKernelGGL(list_combine_kernel, dim3((unsigned)nb), dim3(CB_T), lds, stream,
                       ag_gtab(tag, thi, tlo, tval, trep, ctrl, cap, src), ks, n, to_cols(a), rows);
    return (int)hipGetLastError();
  }
