"""WordCount taskfn (reference: examples/WordCount/taskfn.lua) — one map job
per source file of this framework."""
import os

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FILES = [os.path.join(_ROOT, "runtime", "server.py"), os.path.join(_ROOT, "runtime", "worker.py"),
         os.path.join(_ROOT, "runtime", "job.py"), os.path.join(_ROOT, "utils", "__init__.py")]


def init(arg):
    pass


def taskfn(emit):
    for i, f in enumerate(FILES, 1):
        emit(i, f)
