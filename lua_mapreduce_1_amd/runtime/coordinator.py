"""Client (and launcher) of the native C++ coordinator (``csrc/coord/coord.cpp``).

The coordinator is this framework's replacement for the MongoDB server of the
reference (/root/reference/mapreduce/cnn.lua, task.lua, persistent_table.lua,
GridFS).  A connection string is ``"host:port"``; ``"inproc"`` (or ``None``)
starts — once per process — a coordinator thread on an ephemeral localhost
port and connects to it, which is what single-process runs and tests use.
"""
from __future__ import annotations

import ctypes
import json
import os
import socket
import struct
import threading

from .. import _build

DEFAULT_PORT = 27027

OP = dict(PING=1, TASK_GET=10, TASK_SET=11, TASK_DROP=12, JOB_INSERT=20, JOB_REMOVE_STATUS=21,
          JOB_FAIL_BROKEN=22, JOB_COUNT=23, JOB_CLAIM=24, JOB_UPDATE=25, JOB_GET=26, JOB_LIST=27, JOB_DROP=28,
          JOB_STATS=29, JOB_EXPIRE=30, JOB_CLAIM_WAIT=31, WAIT_CHANGE=32, ERR_INSERT=40, ERR_TAKE=41, BLOB_PUT=50, BLOB_GET=51, BLOB_LIST=52,
          BLOB_DEL=53, BLOB_PUT_MANY=54, BLOB_GET_MANY=55, BLOB_DEL_MANY=56, PT_OPEN=60, PT_UPDATE=61,
          PT_LOCK=62, PT_UNLOCK=63, PT_DROP=64, DB_DROP=70, COLLECTIONS=71, SHUTDOWN=99)

_LIB = None
_LIB_LOCK = threading.Lock()
_INPROC: dict[str, str] = {}


def _lib():
    global _LIB
    with _LIB_LOCK:
        if _LIB is None:
            if not os.path.exists(_build.COORD_LIB):
                _build.build_cxx("coord", "coord", _build.COORD_LIB)
            L = ctypes.CDLL(_build.COORD_LIB)
            L.mrc_start.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p]
            L.mrc_start.restype = ctypes.c_int
            L.mrc_serve_forever.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p]
            L.mrc_serve_forever.restype = ctypes.c_int
            _LIB = L
    return _LIB


def start_local(port: int = 0, host: str = "127.0.0.1", journal: str | None = None) -> str:
    """Start a coordinator thread in this process; returns its connection string."""
    p = _lib().mrc_start(host.encode(), int(port), (journal or "").encode())
    if p <= 0:
        raise RuntimeError(f"coordinator failed to start on {host}:{port}")
    return f"{host}:{p}"


def serve_forever(port: int = DEFAULT_PORT, host: str = "0.0.0.0", journal: str | None = None) -> int:
    return _lib().mrc_serve_forever(host.encode(), int(port), (journal or "").encode())


def resolve(connection_string: str | None) -> str:
    """Map a connection string to host:port, starting an in-process server for
    ``inproc`` / ``None`` (memoised per process)."""
    cs = connection_string or "inproc"
    if cs.startswith("inproc"):
        if cs not in _INPROC:
            _INPROC[cs] = start_local()
        return _INPROC[cs]
    if cs == "localhost":
        return f"127.0.0.1:{DEFAULT_PORT}"
    if ":" not in cs:
        return f"{cs}:{DEFAULT_PORT}"
    return cs


def _enc(x) -> bytes:
    if isinstance(x, bytes):
        return x
    if isinstance(x, float):
        return repr(x).encode()
    return str(x).encode("utf-8", "surrogateescape")


class CoordError(RuntimeError):
    pass


class Client:
    """Blocking request/response client (one socket, thread-safe)."""

    def __init__(self, connection_string: str | None = None, timeout: float | None = 300.0):
        self.address = resolve(connection_string)
        host, port = self.address.rsplit(":", 1)
        self.host, self.port = host, int(port)
        self.timeout = timeout
        self._sock = None
        self._lock = threading.Lock()

    def _connect(self):
        s = socket.create_connection((self.host, self.port), timeout=self.timeout)
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self._sock = s

    def close(self):
        if self._sock is not None:
            try:
                self._sock.close()
            finally:
                self._sock = None

    def _recv(self, n: int) -> bytearray:
        """Exactly n bytes, received straight into one buffer."""
        buf = bytearray(n)
        mv = memoryview(buf)
        got = 0
        while got < n:
            k = self._sock.recv_into(mv[got:], n - got)
            if not k:
                raise ConnectionError("coordinator closed the connection")
            got += k
        return buf

    def request(self, op: str, *fields) -> tuple[int, list[bytes]]:
        parts = [b"", struct.pack("<H", OP[op])]
        for b in map(_enc, fields):
            parts.append(struct.pack("<I", len(b)))
            parts.append(b)
        body_len = sum(len(x) for x in parts)
        parts[0] = struct.pack("<I", body_len)
        msg = b"".join(parts)
        with self._lock:
            for attempt in (0, 1):  # reconnect once (cnn.lua:34-39 auto-reconnect)
                try:
                    if self._sock is None:
                        self._connect()
                    self._sock.sendall(msg)
                    (n,) = struct.unpack("<I", self._recv(4))
                    data = self._recv(n)
                    break
                except (ConnectionError, OSError):
                    self.close()
                    if attempt:
                        raise
        (status,) = struct.unpack_from("<i", data, 0)
        out, p = [], 4
        mv = memoryview(data)
        end = len(data)
        while p < end:
            (ln,) = struct.unpack_from("<I", data, p)
            out.append(bytes(mv[p + 4:p + 4 + ln]))
            p += 4 + ln
        if status < 0:
            raise CoordError(f"coordinator error {status} on {op}")
        return status, out

    # -- convenience -----------------------------------------------------------
    def ping(self) -> bool:
        return self.request("PING", "")[1][0] == b"pong"

    def shutdown(self):
        try:
            self.request("SHUTDOWN", "")
        finally:
            self.close()


# ---------------------------------------------------------------------------
JOB_FIELDS = ("_id", "value", "worker", "tmpname", "status", "repetitions", "creation_time", "started_time",
              "finished_time", "written_time", "broken_time", "cpu_time", "real_time", "heartbeat")


def decode_jobs(fields: list[bytes]) -> list[dict]:
    out = []
    k = len(JOB_FIELDS)
    for i in range(0, len(fields), k):
        f = fields[i:i + k]
        d = {
            "_id": f[0].decode("utf-8", "surrogateescape"),
            "value": json.loads(f[1]) if f[1] else None,
            "worker": f[2].decode(),
            "tmpname": f[3].decode(),
            "status": int(f[4]),
            "repetitions": int(f[5]),
        }
        for name, raw in zip(JOB_FIELDS[6:], f[6:]):
            v = float(raw)
            if name in ("started_time", "written_time") and v < 0:
                continue
            d[name] = v
        out.append(d)
    return out
