"""One map job per file of a split directory (reference: examples/WordCountBig/taskfn.lua,
which lists /home/experimentos/CORPORA/EUROPARL/en-splits/*).  The directory is the
first init argument (default /tmp/lmr_europarl_splits)."""
import glob
import os

DIRECTORY = "/tmp/lmr_europarl_splits"


def init(arg):
    global DIRECTORY
    if arg:
        DIRECTORY = arg[0] if isinstance(arg, (list, tuple)) else arg


def taskfn(emit):
    for i, f in enumerate(sorted(glob.glob(os.path.join(DIRECTORY, "*"))), 1):
        emit(i, f)
