"""Every tunable of the framework in one place, with environment overrides.

The reference has no flag system: its knobs are the constants of
``mapreduce/utils.lua:24-56`` plus the positional CLI arguments
(SURVEY.md §5.6).  Here the user-facing configuration stays the reference's
``server:configure{...}`` table and CLI, and the framework's own knobs — the
reference constants that make sense to change, the device data-plane switches
and the diagnostics — are fields of one frozen dataclass, each with an
``MR_*`` environment override, read once at import.

    python -m lua_mapreduce_1_amd.utils.config      # print every knob, its value and source
"""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass, field


def _flag(v: str) -> bool:
    return v.strip().lower() not in ("", "0", "false", "no", "off")


def _knob(env: str, default, doc: str):
    return field(default=default, metadata={"env": env, "doc": doc})


@dataclass(frozen=True)
class Tunables:
    # -- reference constants (utils.lua:24-56) that are tunable here
    default_sleep: float = _knob("MR_DEFAULT_SLEEP", 1.0, "poll period of server and workers, s (utils.lua:28)")
    long_poll: bool = _knob("MR_LONG_POLL", True,
                            "server/worker: wait for coordinator changes (long-poll claims, change waits) instead "
                            "of sleeping a poll period; the poll period becomes the longest wait")
    job_lease: float = _knob("MR_JOB_LEASE", 120.0,
                             "a RUNNING job whose worker stopped heart-beating this long is re-queued, s (new)")
    fault: str = _knob("MR_FAULT", "",
                       "worker fault injection 'phase:job:action[:times]', e.g. 'map:2:raise:1' (tests)")
    spmd_checkpoint: str = _knob("MR_SPMD_CKPT", "",
                                 "SPMD engine: directory of the iteration manifest (resume after a relaunch)")
    coll_timeout: float = _knob("MR_COLL_TIMEOUT", 600.0,
                                "collective timeout, s: a hung or dead rank fails its peers' collectives")
    spmd_fault: str = _knob("MR_SPMD_FAULT", "",
                            "SPMD fault injection 'iteration:rank:raise|exit[:attempt[:start|shuffle]]': that rank "
                            "fails at the start of that iteration or after its map phase")
    # -- device data plane
    map_sparsity: int = _knob("MR_MAP_SPARSITY", 8,
                              "SPMD fold plane: after a map of at least MR_MAP_SPARSE_MIN_MB of input, later "
                              "maps get a table of this many slots per distinct key (power of two); sparse "
                              "tables probe less and spread the flush's atomics (tools/map_cap_ab.py)")
    map_sparse_min_mb: float = _knob("MR_MAP_SPARSE_MIN_MB", 128.0,
                                     "SPMD fold plane: input MiB per rank and iteration from which map tables "
                                     "are made sparse (MR_MAP_SPARSITY)")
    numa_bind: bool = _knob("MR_NUMA_BIND", True,
                            "SPMD ranks (bench.py, execute_spmd): restrict the rank's CPU threads to the NUMA "
                            "node of its GPU before pinned buffers are allocated (utils/numa.py)")
    pin_exact: bool = _knob("MR_PIN_EXACT", True,
                            "split buffers in exact-size pinned memory (mr_host_alloc) instead of torch's "
                            "power-of-two pinned pool")
    sort_rounds: int = _knob("MR_SORT_ROUNDS", 24,
                             "keys per thread of the onesweep radix tiles of sorts of >= 4 M keys (256 x rounds "
                             "keys per tile; 16, 24 or 32)")
    csv_tiles: int = _knob("MR_CSV_TILES", 0,
                           "fused CSV fold (emit.csv): 8 KiB tiles per workgroup (0 = auto: up to 4 while the "
                           "launch keeps >= 1024 workgroups)")
    csv_mode: int = _knob("MR_CSV_MODE", 0,
                          "fused CSV fold ablation: 0 = normal, 1 = parse only (no insert: wrong results), 2 = no "
                          "LDS combine")
    agg_insert_grid: int = _knob("MR_AGG_INSERT_GRID", 65536,
                                 "general plane: workgroup cap of the per-row table insert (>= 256; one row per "
                                 "thread up to 16 M rows, profiles/r4/agg_grid_ab)")
    recognize_reducers: bool = _knob("MR_RECOGNIZE_REDUCERS", True,
                                     "general plane: a host reducefn / combinerfn that is exactly emit(sum|min|max("
                                     "values)) (or the accumulate loop) runs batched on the device "
                                     "(parallel/recognize.py)")
    const_runs: bool = _knob("MR_CONST_RUNS", True,
                             "general plane, value lists on the GPU: rows that all carry one constant value are "
                             "counted per key (run-length postings) until a row with another value arrives "
                             "(ops/agg.py AggTable.runs)")
    rec_gather_rows: int = _knob("MR_REC_GATHER_ROWS", 256,
                                 "record plane: rows per workgroup batch of the 16-byte row gather (256, or 128: "
                                 "half the LDS image, more workgroups per CU)")
    arena_cap_mb: float = _knob("MR_ARENA_CAP_MB", 0.0,
                                "SPMD: cap of a rank's HBM input arena, MiB (0 = the rank's whole input); a larger "
                                "input is mapped in rounds through a ring of two arenas of this size")
    stream_heap_mb: float = _knob("MR_STREAM_HEAP_MB", 64.0,
                                  "SPMD streaming rounds: HBM heap for the bytes of distinct long keys, MiB")
    record_cap_mb: float = _knob("MR_RECORD_CAP_MB", 0.0,
                                 "SPMD record plane: HBM budget for a rank's rows, MiB (0 = unbounded); more rows "
                                 "spill to host memory and are sorted externally (bucket pass + per-bucket sorts)")
    reduce_cap_mb: float = _knob("MR_REDUCE_CAP_MB", 0.0,
                                 "SPMD list / general planes: HBM budget of one reduce round, MiB (0 = one round); "
                                 "a rank's partitions are ordered and reduced in rounds of at most this many key "
                                 "and value bytes, each round's result moved to host memory")
    fused_tail: bool = _knob("MR_FUSED_TAIL", True, "fused reduce-side tail kernels (tail.hip)")
    single_sync: bool = _knob("MR_SINGLE_SYNC", True,
                              "SPMD fold plane at W > 1: the map's checks ride on the count exchange and the reduce "
                              "tail is launched for a row bound, so an iteration waits on the device twice (count "
                              "exchange, result download) instead of four times")
    pipeline: bool = _knob("MR_PIPELINE", True, "bench/proxies: map of iteration i+1 overlaps the tail of i")
    prefetch_single: bool = _knob("MR_PREFETCH_SINGLE", True, "prefetched inputs: one DMA per iteration")
    sdma_min_mb: float = _knob("MR_SDMA_MIN_MB", 8.0,
                               "result downloads of at least this many MiB go over the SDMA copy engines (ROCr copy "
                               "API, csrc/hip/sdma.hip) after the tail's kernels, not as a runtime blit kernel on "
                               "the CUs beside the next map (0 = never)")
    spin_us: float = _knob("MR_SPIN_US", 2000.0, "host spin on completion words before hipStreamSynchronize, us")
    rec_chunks: int = _knob("MR_REC_CHUNKS", 3,
                            "record plane at W > 1 (R <= W partitions, sampled splitters): rounds of the exchange "
                            "pipelined by key range — every destination's range cut in this many sub-ranges, round "
                            "k's all-to-all overlapping the receive-side sort of round k-1 (0: one exchange, then "
                            "one sort of everything received)")
    exact_alpha: bool = _knob("MR_EXACT_ALPHA", True,
                              "exact key order of 7-bit keys: sort words re-coded to the byte values present "
                              "(5-bit digits for 17-31 values, 6-bit for 32-63: 11-13 radix passes instead of 15)")
    agg_batch: bool = _knob("MR_AGG_BATCH", False,
                            "generic combine kernel: rows for the HBM table probe their home slots in batches of "
                            "four per thread (csrc/hip/hashtab.h gtab_find_or_claim_home) instead of one insert each")
    agg_phases: int = _knob("MR_AGG_PHASES", 1,
                            "generic combine kernel: a thread's 8 rows in 1, 2 or 4 phases (fewer row keys held in "
                            "registers: 79 / 56 / fewer VGPRs, 6 / 7 / more waves per SIMD)")
    rec_ship_keys: bool = _knob("MR_REC_SHIP_KEYS", False,
                                "range-pipelined exchange on the GPU: each round's 32-bit key prefixes travel beside "
                                "its rows (the receive-side sort skips its key pass over the rows; W = 8 proxy: "
                                "-6 % at a 1000 GB/s link model, +3 % at 400, even at 700 — off: one collective per "
                                "round)")
    map_dyn: bool = _knob("MR_MAP_DYN", True,
                          "word-count map kernel: waves take the tile's token list 64 entries at a time from an "
                          "LDS counter (csrc/hip/wordcount3.hip DYN) instead of a fixed stride")
    force_shuffle: bool = _knob("MR_FORCE_SHUFFLE", False,
                                "SPMD: run the W>1 shuffle (pack, count exchange, all-to-all, receive insert) also "
                                "at world size 1 (needs an initialised process group; tests RCCL on one GPU)")
    device_timing: bool = _knob("MR_DEVICE_TIMING", True,
                                "SPMD: HIP events around every map chunk, the shuffle and the tail; job records "
                                "and the stats block report device spans instead of host issue times")
    combine_postings: int = _knob("MR_COMBINE_POSTINGS", 1 << 26,
                                  "general plane, list mode with a combiner: a rank's map table runs the "
                                  "reduce module's combiner over its value lists whenever it holds this many "
                                  "postings (the batched MAX_MAP_RESULT of job.lua:92-96; bounds map memory)")
    # -- diagnostics
    debug_checks: bool = _knob("MR_DEBUG_CHECKS", False, "extra host-side consistency checks (slow)")
    roctx: bool = _knob("MR_ROCTX", False, "roctx ranges around every phase (rocprofv3 --marker-trace)")
    host_timeline: bool = _knob("MR_HOST_TIMELINE", False, "record phase ranges with perf_counter (trace.LOG)")
    host_timeline_hip: bool = _knob("MR_HOST_TIMELINE_HIP", False, "... and every native call")
    wait_log: bool = _knob("MR_WAIT_LOG", False, "log every host wait (ops._hip.WAIT_LOG)")

    @classmethod
    def from_env(cls, env=None) -> "Tunables":
        env = os.environ if env is None else env
        kw = {}
        for f in dataclasses.fields(cls):
            v = env.get(f.metadata["env"])
            if v is None:
                continue
            if f.type in ("bool", bool):
                kw[f.name] = _flag(v)
            elif f.type in ("int", int):
                kw[f.name] = int(v)
            elif f.type in ("float", float):
                kw[f.name] = float(v)
            else:
                kw[f.name] = v
        return cls(**kw)

    def describe(self) -> str:
        rows = []
        for f in dataclasses.fields(self):
            env = f.metadata["env"]
            src = "env" if env in os.environ else "default"
            rows.append(f"{f.name:18s} {env:22s} {str(getattr(self, f.name)):10s} {src:7s} {f.metadata['doc']}")
        return "\n".join(rows)


TUNABLES = Tunables.from_env()


if __name__ == "__main__":
    print(TUNABLES.describe())
