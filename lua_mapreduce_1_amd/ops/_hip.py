"""ctypes binding of ``_lib/libmrhip.so`` (the gfx950 HIP kernels).

Every entry point takes raw device pointers of torch-owned tensors and the
current HIP stream; nothing inside allocates or synchronises, so the calls are
hipGraph-capturable.  On a machine with a GPU the library is mandatory: if it
cannot be loaded, :func:`lib` raises instead of silently falling back.
"""
from __future__ import annotations

import ctypes
import os
import threading
import time

import torch  # noqa: F401  (must be imported first: provides libamdhip64.so.7)

from .. import _build
from ..utils.config import TUNABLES

_LOCK = threading.Lock()
_LIB = None

_u64 = ctypes.c_uint64
_i32 = ctypes.c_int
_u32 = ctypes.c_uint32
_p = ctypes.c_void_p

_SIGS = {
    "mr_count_tokens": [_p, _u64, _u64, _p, _p],
    "mr_wc_map3": [_p, _u64, _u64, _p, _p, _p, _p, _p, _p, _u64, _p, _p, _p, _u64, _p, _p],
    "mr_insert_received": [_p, _u64, _p, _u32, _p, _p, _p, _p, _p, _p, _u64, _i32, _i32, _p, _p],
    "mr_memcpy_async": [_p, _p, _u64, _i32, _p],
    "mr_d2h_async": [_p, _p, _u64, _p],
    "mr_h2d_pull": [_p, _p, _u64, _i32, _p],
    "mr_signal_host": [_p, _u32, _p],
    "mr_tail_run": [_p, _p, _p, _p, _p, _p, _u64, _u64, _u32, _p, _p, _p, _u64, _p, _p, ctypes.c_longlong, _u64,
                    _i32, _p],
    "mr_tokenize": [_p, _u64, _u64, _u64, _p, _p, _p, _u64, _p, _p],
    "mr_hash_agg": [_p, _p, _p, _p, _u64, _u64, _i32, _p, _p, _p, _p, _p, _p, _u64, _p, _p],
    "mr_table_compact": [_p, _p, _p, _p, _p, _p, _u64, _p, _p, _p, _p, _p, _p, _p],
    "mr_gather_aos4": [_p, _u64, _p, _p, _p, _p, _p, _p, _p],
    "mr_rec_gather_set_rows": [_i32],
    "mr_csv_fold": [_p, _p, _p, _p, _p, _p, _u64, _p, _p, _u64, _u64, _p, _p, _p, _p],
    "mr_key_word": [_p, _p, _p, _p, _u64, _u32, _p, _p],
    "mr_key_meta": [_p, _p, _p, _u64, _p, _u32, _p, _p, _p, _p, _p, _p, _p],
    "mr_pack_alpha": [_p, _u64, _p, _u32, _u32, _p, _p],
    "mr_gather_key_bytes": [_p, _p, _p, _p, _u64, _p, _p, _u64, _p],
    "mr_exclusive_scan_u32": [_p, _p, _u64, _p, _p, _p],
    "mr_exclusive_scan_i64": [_p, _p, _u64, _p, _p, _p],
    "mr_gather_u64": [_p, _p, _p, _u64, _p],
    "mr_radix_ghist8": [_p, _u64, _p, _i32, _p],
    "mr_radix_onesweep_u32v": [_p, _p, _p, _p, _u64, _i32, _p, _p, _p, _u32, _p, _i32, _p],
    "mr_iota_u32": [_p, _u64, _p],
    "mr_segment_heads": [_p, _p, _u64, _p, _p],
    "mr_segment_fold": [_p, _p, _p, _u64, _i32, _p, _p],
    "mr_segment_keys": [_p, _p, _p, _p, _p, _u64, _p, _p, _p, _p, _p],
    "mr_bincount": [_p, _u64, _u32, _p, _p],
    "mr_composite_key": [_p, _p, _u64, _p, _p],
    "mr_copy_to_host": [_p, _p, _p, _u64, _u64, _p],
    "mr_tie_fixup": [_p, _p, _p, _p, _p, _p, _u64, _p, _p, _p, _p],
    "mr_gather_cols": [_p, _u64, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p],
    "mr_mlp_grad": [_p, _p, _p, _i32, _i32, _i32, _i32, _p, _p, _p, _p, _p, _i32, _p],
    "mr_mlp_sgd": [_p, _p, _p, _i32, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float, _i32, _i32,
                   _i32, _p],
    "mr_mlp_param_count": [_i32, _i32, _i32],
    "mr_count_newlines": [_p, _u64, _u64, _p, _p, _p],
    "mr_ii_map": [_p, _u64, _u64, _u64, _p, _p, _p, _p, _p, _p, _p, _p, _p, _u64, _u32, _p, _p, _u64, _p, _p],
    "mr_ii_advance": [_p, _p, _p],
    "mr_ii_add_dest": [_p, _u64, _p, _u32, _u64, _u32, _p],
    "mr_ii_unique_tiles": [_u64],
    "mr_ii_unique_count": [_p, _u64, _p, _p],
    "mr_ii_unique_scatter": [_p, _u64, _p, _p, _p],
    "mr_ii_group_count": [_p, _u64, _u32, _i32, _p, _p],
    "mr_ii_group_scatter": [_p, _u64, _u32, ctypes.c_longlong, _u64, _i32, _p, _p, _p, _p, _p],
    "mr_ii_insert_slots": [_p, _p, _p, _p, _p, _p, _u64, _p, _p, _p, _u64, _p, _p, _p],
    "mr_ii_seg_gather": [_p, _p, _p, _u64, _u64, _u64, _u64, _p, _p, _p],
    "mr_ts_gen": [_p, _u64, _u64, _u64, _p],
    "mr_ts_keys": [_p, _u64, _p, _p, _p, _p],
    "mr_ts_checksum": [_p, _u64, _p, _p],
    "mr_ts_unsorted": [_p, _p, _u64, _p, _p],
    "mr_pack_by_dest": [_p, _p, _p, _p, _p, _u64, _u32, _p, _p, _p, ctypes.c_longlong, _p, _p, _i32, _p],
    "mr_fix_loc": [_p, _u64, _p, _p, _u32, _p, _p],
    "mr_tail_compact": [_p, _p, _p, _p, _p, _p, _u64, _u32, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _u64, _u64,
                        _i32, _p, _p],
    "mr_tail_bhist_bytes": [_u64],
    "mr_tail_gather": [_p, _u64, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p],
    "mr_tail_pack": [_p, _p, _u64, _p, _u32, _p, _p, _p, _p],
    "mr_sort_debug_fail": [_i32],
    "mr_sort_set_rounds": [_i32],
    "mr_sort_set_rounds32": [_i32],
    "mr_onesweep_tiles": [_u64],
    "mr_set_long_mask_wc3": [_u64],
    "mr_set_long_mask_keyops": [_u64],
    "mr_set_long_mask_invidx": [_u64],
    "mr_tail_pack_bytes": [_u64, _u32],
    "mr_tail_ws_layout": [_u64, _u32, _u64, _u64, ctypes.POINTER(ctypes.c_uint64)],
    "mr_table_reset": [_p, _p, _p, _u64, ctypes.c_longlong, _p],
    "mr_table_rehome": [_p, _u64, _p, _u64, _u64, _p, _u64, _p],
    "mr_scan_partials_len": [_u64],
    "mr_radix_onesweep_k32": [_p, _p, _p, _p, _u64, _i32, _p, _p, _p, _u32, _p, _i32, _p],
    "mr_rec_keys32": [_p, _u64, _i32, _i32, _p, _p, _p],
    "mr_rec_keys": [_p, _u64, _i32, _i32, _p, _p, _p],
    "mr_rec_tie_fixup": [_p, _p, _p, _u64, _i32, _i32, _p, _p, _u64, _p],
    "mr_rec_gather": [_p, _u64, _p, _u64, _i32, _p, _i32, _p],
    "mr_rec_dest32": [_p, _u64, _p, _u32, _p, _p],
    "mr_rec_bucket32": [_p, _u64, _p, _u32, _u32, _u32, _p, _p, _p],
    "mr_rec_sample32": [_p, _u64, _u32, _u64, _p, _p],
    "mr_rec_hist32": [_p, _u64, _p, _p],
    "mr_rec_pick": [_p, _u64, _u32, _p, _p],
    "mr_rec_xchg": [_p, _u32, _u32, ctypes.c_longlong, _p, _p, _p, _p],
    "mr_agg_insert": [_p, _p, _p, _p, _p, _p, _u64, _p, _p, _p, _p, _u64, _p, _p, _p, _u64, _u64, _p, _p],
    "mr_slot_compact": [_p, _p, _p, _p, _p, _p, _u64, _p, _p, _p, _p, _p, _p],
    "mr_col_fill": [_p, _u64, ctypes.c_longlong, _i32, _p],
    "mr_set_long_mask_generic": [_u64],
    "mr_text_tiles": [_u64],
    "mr_text_count": [_p, _u64, _i32, _u32, _p, _p, _p],
    "mr_text_emit": [_p, _u64, _i32, _u32, _p, _u64, _p, _p, _p, _p, _p],
    "mr_text_field": [_p, _p, _p, _u64, _u32, _i32, _p, _p, _p],
    "mr_text_parse_f64": [_p, _p, _p, _u64, _p, _p, _p],
    "mr_text_parse_i64": [_p, _p, _p, _u64, _p, _p, _p],
    "mr_rec_tie_ws_words": [_u64, _u64],
    "mr_exact_hash": [_p, _p, _p, _p, _u64, _p, _p],
    "mr_exact_fix": [_p, _p, _u64, _p, _p, _p, _p, _p, _p, _p, _p],
    "mr_seg_reduce": [_p, _u64, _p, _u64, _i32, _i32, _p, _p],
    "mr_posting_keys": [_p, ctypes.c_longlong, _p, ctypes.c_longlong, ctypes.c_longlong, _p, _p, _p],
    "mr_csv_set_config": [_i32, _i32],
    "mr_agg_set_insert_grid": [_i32],
    "mr_small_d2h": [_p, _p, _p, _i32, _p, _p, _u32, _p],
    "mr_compact_pack_ws_bytes": [_u64, _u32],
    "mr_compact_pack": [_p, _p, _p, _p, _p, _p, _u64, _u32, _u32, _p, _p, _p, _u64, _p, ctypes.c_longlong, _p, _u32,
                        _p, _p],
    "mr_sdma_available": [],
    "mr_sdma_d2h": [_p, _p, _p, _i32],
    "mr_sdma_d2h_begin": [_p, _p, _p, _i32, _p],
    "mr_sdma_wait": [_u64],
    "mr_ipc_alloc": [_u64, ctypes.POINTER(ctypes.c_void_p)],
    "mr_ipc_free": [_p],
    "mr_ipc_handle": [_p, _p],
    "mr_ipc_open": [_p, ctypes.POINTER(ctypes.c_void_p)],
    "mr_ipc_close": [_p],
    "mr_gather_copy": [_p, _u32, _u64, _p],
    "mr_gather_copy_chunk": [],
    "mr_mrc1_decode": [_p, _p, _u32, _u64, _p, _p, _p, _p, _p],
    "mr_wc3_set_dyn": [_i32],
    "mr_agg_set_batch": [_i32],
    "mr_agg_set_phases": [_i32],
}
_RESTYPE_U64 = {"mr_compact_pack_ws_bytes", "mr_ii_unique_tiles", "mr_text_tiles", "mr_scan_partials_len", "mr_tail_pack_bytes", "mr_tail_ws_layout",
                "mr_tail_bhist_bytes", "mr_onesweep_tiles", "mr_rec_tie_ws_words", "mr_sdma_d2h_begin",
                "mr_gather_copy_chunk"}


def lib():
    """Load (building first if needed) the HIP kernel library."""
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is not None:
            return _LIB
        path = _build.build_hip()  # no-op unless a source is newer than the .so
        L = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        for name, args in _SIGS.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = _u64 if name in _RESTYPE_U64 else _i32
        L.mr_host_alloc_coherent.argtypes = [_u64]
        L.mr_host_alloc_coherent.restype = _p
        L.mr_host_alloc.argtypes = [_u64]
        L.mr_host_alloc.restype = _p
        L.mr_host_free.argtypes = [_p]
        L.mr_host_free.restype = _i32
        if L.mr_sort_set_rounds(TUNABLES.sort_rounds) != 0:
            raise ValueError(f"MR_SORT_ROUNDS={TUNABLES.sort_rounds}: must be 16, 24 or 32")
        if L.mr_csv_set_config(TUNABLES.csv_tiles, TUNABLES.csv_mode) != 0:
            raise ValueError(f"MR_CSV_TILES={TUNABLES.csv_tiles} / MR_CSV_MODE={TUNABLES.csv_mode}: 0..64 / 0..2")
        if L.mr_agg_set_insert_grid(TUNABLES.agg_insert_grid) != 0:
            raise ValueError(f"MR_AGG_INSERT_GRID={TUNABLES.agg_insert_grid}: must be >= 256")
        L.mr_wc3_set_dyn(1 if TUNABLES.map_dyn else 0)
        L.mr_agg_set_batch(1 if TUNABLES.agg_batch else 0)
        L.mr_agg_set_phases(TUNABLES.agg_phases if TUNABLES.agg_phases in (1, 2, 4) else 1)
        if L.mr_rec_gather_set_rows(TUNABLES.rec_gather_rows) != 0:
            raise ValueError(f"MR_REC_GATHER_ROWS={TUNABLES.rec_gather_rows}: must be 128 or 256")
        _LIB = L
    return _LIB


_LONG_MASK_SETTERS = ("mr_set_long_mask_wc3", "mr_set_long_mask_keyops", "mr_set_long_mask_invidx",
                      "mr_set_long_mask_generic")


def set_long_mask(mask: int) -> None:
    """Long-key hash mask of every kernel translation unit (debug knob; see
    ops.keys.set_long_hash_bits)."""
    for name in _LONG_MASK_SETTERS:
        call(name, mask)


_AVAILABLE: list = []


def available() -> bool:
    """torch.cuda.is_available(), asked once (each call costs milliseconds
    on this stack)."""
    if not _AVAILABLE:
        _AVAILABLE.append(torch.cuda.is_available())
    return _AVAILABLE[0]


def ptr(t):
    if t is None:
        return None
    if not t.is_contiguous():
        # kernels index raw memory: a strided view would be read as garbage
        raise ValueError("HIP kernels need contiguous tensors")
    return ctypes.c_void_p(t.data_ptr())


def stream(device=None):
    """Raw hipStream_t of the current stream (torch's raw-stream accessor:
    torch.cuda.current_stream() builds a Stream object, ~5 us per call)."""
    if device is None:
        idx = torch.cuda.current_device()
    elif isinstance(device, int):
        idx = device
    else:
        idx = device.index if device.index is not None else torch.cuda.current_device()
    return ctypes.c_void_p(torch._C._cuda_getCurrentRawStream(idx))


def stream_ptr(s) -> ctypes.c_void_p:
    """Raw hipStream_t of a torch stream object."""
    return ctypes.c_void_p(s.cuda_stream)


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"HIP kernel launch failed in {what}: error {rc}")


def call(name: str, *args) -> None:
    if _TLOG is not None:
        t = time.perf_counter()
        rc = getattr(lib(), name)(*args)
        _TLOG.append(("hip:" + name, t, time.perf_counter()))
    else:
        rc = getattr(lib(), name)(*args)
    check(rc, name)


_TLOG = None
if TUNABLES.host_timeline_hip:  # every native call in the host timeline (utils/trace.LOG)
    from ..utils import trace as _trace
    _TLOG = _trace.LOG


class _HostFlags:
    """Completion flags in coherent pinned memory, one word per stream."""

    def __init__(self):
        import numpy as np
        self.nslots = 1024
        p = lib().mr_host_alloc_coherent(4 * self.nslots)
        if not p:
            raise RuntimeError("hipHostMalloc of the completion flags failed")
        self.base = p
        self.words = np.ctypeslib.as_array((ctypes.c_uint32 * self.nslots).from_address(p))
        self.slot: dict = {}
        self.seq = 0


_FLAGS = None
SPIN_S = TUNABLES.spin_us * 1e-6


def wait_stream(device=None) -> None:
    """Wait for the work queued so far on the current stream: a one-thread
    kernel behind it stores a sequence number into coherent pinned memory
    (mr_signal_host) and the host spins on that word — no sleep/interrupt
    wake-up.  After ``MR_SPIN_US`` (2000) of spinning, falls back to
    hipStreamSynchronize (which also reports a failed kernel).
    ``MR_SPIN_US=0``: always hipStreamSynchronize."""
    if SPIN_S <= 0:
        WAITS[0] += 1
        torch.cuda.current_stream(device).synchronize()
        return
    flag, k, seq = next_signal(device)
    call("mr_signal_host", flag, seq, stream(device))
    spin(k, seq, device)


def next_signal(device=None):
    """(flag address, slot, sequence number) for a completion signal queued
    on the current stream: the caller's kernel stores ``seq`` there (the
    signal kernel, or a download that signals itself: mr_small_d2h)."""
    global _FLAGS
    if _FLAGS is None:
        _FLAGS = _HostFlags()
    F = _FLAGS
    sp = stream(device)
    k = F.slot.get(sp.value)
    if k is None:
        k = F.slot[sp.value] = len(F.slot) % F.nslots
    F.seq = (F.seq + 1) & 0x7FFFFFFF or 1
    return ctypes.c_void_p(F.base + 4 * k), k, F.seq


def _done(w: int, seq: int) -> bool:
    # signals of one stream complete in order: a later one seen means ours is done
    return ((int(w) - seq) & 0x7FFFFFFF) < 0x40000000


def spin(k: int, seq: int, device=None) -> None:
    """Host wait for the signal (slot k, seq): spin on the word, then after
    MR_SPIN_US fall back to synchronising the current stream."""
    WAITS[0] += 1
    w = _FLAGS.words
    if WAIT_LOG is not None:
        t_a = time.perf_counter()
    if not _done(w[k], seq):
        t_end = time.perf_counter() + SPIN_S
        n = 0
        while not _done(w[k], seq):
            n += 1
            if (n & 255) == 0 and time.perf_counter() > t_end:
                torch.cuda.current_stream(device).synchronize()
                break
    if WAIT_LOG is not None:
        WAIT_LOG.append((t_a, time.perf_counter(), _done(w[k], seq)))


WAITS = [0]  # host waits on a stream so far (tests count them per iteration)
WAIT_LOG = [] if TUNABLES.wait_log else None  # (start, end, flag seen) of each wait_stream
