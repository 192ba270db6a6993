    def _alloc_cols(self, cols: list) -> list:
        """The physical columns on the GPU.  With more than one column, all
        of 8 bytes, they are one row per slot (4 or 8 words: a row never
        straddles a 64-byte line), so the folds of a key touch one line of
        memory instead of one per column (MR_AGG_ROWS); otherwise one array
        per column."""
        k = len(cols)
        if TUNABLES.agg_rows and k > 1 and all(dt in ("i64", "f64") for dt, _op, _i in cols):
            self.cstride = 4 if k <= 4 else 8
            buf = torch.empty(self.cap, self.cstride, dtype=torch.int64, device=self.device)
            return [buf[:, j].view(DTYPES[dt]) for j, (dt, _op, _i) in enumerate(cols)]
        return [torch.empty(self.cap, dtype=DTYPES[dt], device=self.device) for dt, _op, _i in cols]

