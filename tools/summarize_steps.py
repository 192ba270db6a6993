#!/usr/bin/env python
"""Summaries of a tools/run_steps.sh output directory: each step's rc, and
the headline fields of the JSON lines its log printed (ms_per_step / median /
valid flags), one line per step.

    python tools/summarize_steps.py gpurun_out/r6/s12
"""
import json
import os
import sys

KEYS = ("ms_per_step", "median", "min", "valid", "validated_full", "sorted", "per_key_valid", "valid_runs",
        "server_time_s_median", "map_ms_plain_min", "phases_ms")


def main(d: str) -> None:
    steps = open(os.path.join(d, "steps.txt")).read().split("\n") if os.path.exists(os.path.join(d, "steps.txt")) \
        else []
    for ln in steps:
        if not ln.startswith("step "):
            continue
        name = ln.split()[1]
        vals = {}
        try:
            for row in open(os.path.join(d, name + ".log"), errors="replace"):
                row = row.strip()
                if row.startswith("{"):
                    try:
                        j = json.loads(row)
                    except ValueError:
                        continue
                    vals.update({k: j[k] for k in KEYS if k in j})
                    if "config" in j and isinstance(j["config"], dict):
                        vals.update({k: j["config"][k] for k in KEYS if k in j["config"]})
                elif " passed" in row or " failed" in row:
                    vals["pytest"] = row
        except OSError:
            pass
        print(ln, json.dumps(vals))


if __name__ == "__main__":
    main(sys.argv[1])
