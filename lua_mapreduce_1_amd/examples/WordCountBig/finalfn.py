"""Summarising finalfn for big runs: total/distinct counts instead of printing
every word (the reference's BIG run redirects the full listing to a file)."""
import sys

TOTAL = 0
DISTINCT = 0


def init(arg):
    pass


def finalfn(pairs_iterator):
    global TOTAL, DISTINCT
    TOTAL = DISTINCT = 0
    for _key, values in pairs_iterator:
        TOTAL += values[0]
        DISTINCT += 1
    sys.stderr.write(f"# words {TOTAL} distinct {DISTINCT}\n")
    return True
