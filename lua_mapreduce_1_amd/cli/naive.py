"""Naive single-process word count oracle (reference: misc/naive.lua).

    cat files... | python -m lua_mapreduce_1_amd.cli.naive   ->  "count word" lines
"""
from __future__ import annotations

import sys


def count(stream) -> dict:
    vocab: dict = {}
    for line in stream:
        for w in line.split():
            vocab[w] = vocab.get(w, 0) + 1
    return vocab


def main() -> int:
    out = sys.stdout.buffer
    for w, v in count(sys.stdin.buffer).items():
        out.write(b"%d %s\n" % (v, w))
    return 0


if __name__ == "__main__":
    sys.exit(main())
