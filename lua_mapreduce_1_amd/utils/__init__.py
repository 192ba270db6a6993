"""Constants, enums and helpers shared by every layer.

Reference: /root/reference/mapreduce/utils.lua:24-56 (constants/enums) and
:62-430 (helpers).  The MongoDB-specific helpers (connect, GridFS line
iterator) are replaced by the coordinator client (:mod:`..runtime.cnn`) and the
storage router (:mod:`..runtime.fs`); the Lua-literal serializer is kept for
text-compatible output, while intermediate data uses a data-only binary codec
(:mod:`.codec`) instead of executable ``return k,{v}`` lines.
"""
from __future__ import annotations

import builtins
import json
import math
import os
import shutil
import socket
import tempfile
import time as _time
from typing import Any, Callable, Iterable, Iterator

from .config import TUNABLES
from .heap import heap  # noqa: F401


_VERSION = "0.3"
_NAME = "mapreduce.utils"

DEFAULT_RW_TIMEOUT = 300          # seconds
DEFAULT_SLEEP = TUNABLES.default_sleep  # seconds (poll period; MR_DEFAULT_SLEEP)
DEFAULT_MICRO_SLEEP = 0.1
DEFAULT_HOSTNAME = "<unknown>"
DEFAULT_TMPNAME = "<NONE>"
DEFAULT_DATE = 0


class STATUS:  # noqa: N801  (job status, utils.lua:33-40)
    WAITING = 0
    RUNNING = 1
    BROKEN = 2
    FINISHED = 3
    WRITTEN = 4
    FAILED = 5


class TASK_STATUS:  # noqa: N801  (task status, utils.lua:41-46)
    WAIT = "WAIT"
    MAP = "MAP"
    REDUCE = "REDUCE"
    FINISHED = "FINISHED"


MAX_IDLE_COUNT = 5
MAX_WORKER_RETRIES = 3
MAX_JOB_RETRIES = 3
MAX_PENDING_INSERTS = 50000
MAX_IT_WO_CGARBAGE = 5000
MAX_TIME_WO_CGARBAGE = 60
MAX_MAP_RESULT = 5000
MAX_TASKFN_VALUE_SIZE = 16 * 1024
GRP_TMP_DIR = os.path.join(tempfile.gettempdir(), "grouped")
# new in this framework: liveness lease for RUNNING jobs (reference has none,
# SURVEY.md §5.3); a RUNNING job whose worker stops heart-beating for this long
# is re-queued as BROKEN.
JOB_LEASE_SECONDS = TUNABLES.job_lease  # MR_JOB_LEASE


def get_hostname() -> str:
    return socket.gethostname()


def sleep(n: float) -> None:
    _time.sleep(n)


def time() -> float:
    return _time.time()


def make_job(key, value) -> dict:
    """Job document (utils.lua:87-98)."""
    if key is None or value is None:
        raise ValueError("Needs a key and a value")
    return {
        "_id": key_to_id(key),
        "value": value,
        "worker": DEFAULT_HOSTNAME,
        "tmpname": DEFAULT_TMPNAME,
        "creation_time": time(),
        "status": STATUS.WAITING,
        "repetitions": 0,
    }


def key_to_id(key) -> str:
    """``tostring(key)`` of the reference (integral floats print as ints)."""
    if isinstance(key, float) and key.is_integer():
        return str(int(key))
    if isinstance(key, bytes):
        return key.decode("utf-8", "surrogateescape")
    return str(key)


# ---------------------------------------------------------------------------
# Lua-literal serialization (utils.lua:100-120) — text-compatible output.

def _lua_number(x) -> str:
    if isinstance(x, bool):
        return "true" if x else "false"
    if isinstance(x, int):
        return str(x)
    if math.isinf(x):
        return "1/0" if x > 0 else "-1/0"
    if math.isnan(x):
        return "0/0"
    if x.is_integer() and abs(x) < 1e15:
        return str(int(x))
    return "%.14g" % x


def lua_quote(s) -> str:
    """``string.format("%q", s)`` of Lua 5.2 (newline escaped as ``\\n``)."""
    if isinstance(s, str):
        b = s.encode("utf-8", "surrogateescape")
    else:
        b = bytes(s)
    out = ['"']
    n = len(b)
    for i, c in enumerate(b):
        if c == 34:
            out.append('\\"')
        elif c == 92:
            out.append("\\\\")
        elif c == 10:
            out.append("\\n")
        elif c == 13:
            out.append("\\r")
        elif c == 0:
            nxt = b[i + 1] if i + 1 < n else None
            out.append("\\000" if nxt is not None and 48 <= nxt <= 57 else "\\0")
        elif c < 32 or c == 127:
            nxt = b[i + 1] if i + 1 < n else None
            out.append("\\%03d" % c if nxt is not None and 48 <= nxt <= 57 else "\\%d" % c)
        else:
            out.append(chr(c) if c < 128 else bytes([c]).decode("latin-1"))
    out.append('"')
    return "".join(out)


def escape(v) -> str:
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return _lua_number(v)
    if isinstance(v, (str, bytes)):
        return lua_quote(v)
    if isinstance(v, (list, builtins.tuple)) and not isinstance(v, str):
        return "tuple{ " + ", ".join(escape(x) for x in v) + " }"
    return str(v)


def serialize_table_ipairs(t: Iterable) -> str:
    return "{" + ",".join(escape(v) for v in t) + "}"


# ---------------------------------------------------------------------------
# Total order over keys (numbers < strings < tuples), the deterministic
# analogue of Lua's `<` used by keys_sorted (utils.lua:123-128).

def sort_key(k):
    if isinstance(k, bool):
        return (0, int(k))
    if isinstance(k, (int, float)):
        return (0, k)
    if isinstance(k, str):
        return (1, k.encode("utf-8", "surrogateescape"))
    if isinstance(k, bytes):
        return (1, k)
    if isinstance(k, (builtins.tuple, list)):
        return (2, len(k), builtins_tuple_map(sort_key, k))
    return (3, str(k))


def builtins_tuple_map(f, seq):
    return builtins.tuple(f(x) for x in seq)


def keys_sorted(result: dict) -> list:
    return sorted(result.keys(), key=sort_key)


def merge_iterator(fs, filenames: list[str], make_lines_iterator: Callable[[str], Iterator]):
    """k-way merge of key-sorted runs, concatenating values of equal keys.

    Reference: utils.lua:206-271 (heap of {k, v, line, which}).  Each input
    iterator yields ``(key, [values])`` records in ``sort_key`` order; the
    output yields ``(key, values)`` with values concatenated in file order.
    """
    iters = [make_lines_iterator(name) for name in filenames]
    queue = heap(lambda a, b: (a[0], a[2]) < (b[0], b[2]))

    def take_next(which: int):
        it = iters[which]
        if it is None:
            return
        rec = next(it, None)
        if rec is None:
            iters[which] = None
            return
        k, v = rec
        queue.push((sort_key(k), k, which, list(v)))

    for i in range(len(iters)):
        take_next(i)
    while not queue.empty():
        sk, key, which, result = queue.top()
        queue.pop()
        take_next(which)
        while not queue.empty() and queue.top()[0] == sk:
            _, _, w2, v2 = queue.top()
            queue.pop()
            take_next(w2)
            result.extend(v2)
        yield key, result


def get_storage_from(s: str | None, new: bool = False) -> tuple[str, str]:
    """Parse ``"name[:/abs/path]"`` (utils.lua:273-285)."""
    s = s or "gridfs"
    if ":" in s and s.split(":", 1)[1].startswith("/"):
        storage, path = s.split(":", 1)
        return storage, path
    if not new:
        raise ValueError(f"Given incorrect storage {s}")
    storage = s.split(":", 1)[0]
    fd, path = tempfile.mkstemp(prefix="lua_")
    os.close(fd)
    os.remove(path)
    return storage, path


def remove(filename: str) -> bool:
    try:
        if os.path.isdir(filename) and not os.path.islink(filename):
            shutil.rmtree(filename)
        else:
            os.remove(filename)
        return True
    except FileNotFoundError:
        return False


def rename(old: str, new: str) -> bool:
    os.replace(old, new)
    return True


def clear_table(t) -> None:
    t.clear()


def copy_table_ipairs(dst: list, src: list) -> None:
    dst[:] = list(src)


def assert_check(value) -> None:
    """Check that a value is JSON compatible (utils.lua:313-333)."""
    if isinstance(value, dict):
        str_keys = [isinstance(k, str) for k in value]
        if any(str_keys) and not all(str_keys):
            raise ValueError("Impossible to mix not string keys with string keys")
        for k, v in value.items():
            assert_check(v)
    elif isinstance(value, (list, builtins.tuple)):
        for v in value:
            assert_check(v)
    elif callable(value):
        raise ValueError("Impossible to assign a function in a JSON table")
    elif not isinstance(value, (str, int, float, bool, type(None), bytes)):
        raise ValueError(f"Impossible to assign a {type(value).__name__} in a JSON table")


def tojson(v) -> str:
    return json.dumps(v, default=lambda o: list(o) if isinstance(o, (builtins.tuple, set)) else str(o))


def utest(connection_string=None) -> None:
    """utils.lua:340-406: hostname/time, Lua-literal serialization golden
    strings, the GridFS line iterator, a golden k-way merge of two sorted
    runs, storage-spec parsing, rename/remove, clear/copy table."""
    from ..runtime import codec
    from ..runtime.cnn import cnn as cnn_cls
    assert isinstance(get_hostname(), str)
    assert abs(time() - _time.time()) < 5
    assert escape(120) == "120"
    assert escape("30") == '"30"'
    assert escape("30\n") == '"30\\n"'
    assert serialize_table_ipairs([1, 2, 3, "hola"]) == '{1,2,3,"hola"}'
    assert serialize_table_ipairs(keys_sorted({"c": 1, "a": 2, "b": 3})) == '{"a","b","c"}'
    g = cnn_cls(connection_string, "test").gridfs()
    lines = [b"first line", b"second", b"third longer line", b"a"]
    g.remove_file("lines")
    g.store_data(b"\n".join(lines), "lines")
    assert list(g.lines("lines")) == lines
    f1 = [(1, [1, 1]), (2, [1]), (3, [1])]
    f2 = [(1, [1, 1, 1, 1]), (3, [1]), (4, [1])]
    for name, recs in (("f1", f1), ("f2", f2)):
        g.remove_file(name)
        g.store_data(codec.encode_records(recs), name)
    got = list(merge_iterator(g, ["f1", "f2"], lambda n: codec.decode_records(g.get(n))))
    assert got == [(1, [1] * 6), (2, [1]), (3, [1, 1]), (4, [1])], got
    for storage in ("gridfs", "sshfs", "shared"):
        for path in ("", ":/tmp/dir"):
            a, b = get_storage_from(storage + path, True)
            assert a == storage and b and (path == "" or ":" + b == path)
    fd1, tmp1 = tempfile.mkstemp()
    os.close(fd1)
    tmp2 = tmp1 + ".renamed"
    assert rename(tmp1, tmp2)
    assert remove(tmp2)
    t = {1: 1, 2: 3, "a": 4, "b": 5}
    clear_table(t)
    assert not t
    src = [1, 2, 3, 4]
    dst1, dst2 = [5, 6, 7], [5, 6, 7, 8, 9, 10]
    copy_table_ipairs(dst1, src)
    copy_table_ipairs(dst2, src)
    assert dst1 == src and dst2 == src
