"""Summarising finalfn for big runs: total/distinct counts instead of printing
every word (the reference's BIG run redirects the full listing to a file).

``MR_FINAL_DUMP=<path>``: every (key bytes, count) pair is also written there
(msgpack), so a harness can check each word against its oracle
(tools/bench_server_worker.py)."""
import os
import sys

TOTAL = 0
DISTINCT = 0


def init(arg):
    pass


def finalfn(pairs_iterator):
    global TOTAL, DISTINCT
    TOTAL = DISTINCT = 0
    dump = os.environ.get("MR_FINAL_DUMP")
    keep = [] if dump else None
    for key, values in pairs_iterator:
        TOTAL += values[0]
        DISTINCT += 1
        if keep is not None:
            kb = key.encode("utf-8", "surrogateescape") if isinstance(key, str) else bytes(key)
            keep.append((kb, int(values[0])))
    if keep is not None:
        import msgpack
        tmp = dump + ".tmp"
        with open(tmp, "wb") as f:
            f.write(msgpack.packb(keep, use_bin_type=True))
        os.replace(tmp, dump)
    sys.stderr.write(f"# words {TOTAL} distinct {DISTINCT}\n")
    return True
