"""Text scanning and parsing for user device map functions (HIP kernels in
``csrc/hip/text.hip``; NumPy on CPU tensors — the executable specification).

A ``device_mapfn`` picks its keys and values out of the staged input bytes
with these plus ordinary torch ops, then hands them to ``emit.spans`` (see
parallel/generic.py).  They replace the reference's Lua string functions in
user map code: ``line:gmatch("[^%s]+")`` (examples/WordCount/mapfn.lua:5),
``io.lines`` (mapfn.lua:4) and ``tonumber``.

Every function returns tensors on the device of ``text``; positions are byte
offsets into ``text`` (int64) and lengths are int32, in text order.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _hip
from .keys import _WS_TABLE


def _np(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().numpy()


def _scan(text: torch.Tensor, mode: int, byte: int, want_len: bool, want_line: bool = False):
    """(positions, lengths | None, line numbers | None) of the items."""
    n = text.numel()
    d = text.device
    if n == 0:
        z = torch.zeros(0, dtype=torch.int64, device=d)
        return z, (torch.zeros(0, dtype=torch.int32, device=d) if want_len else None), (z.clone() if want_line else None)
    if text.is_cuda:
        from .primitives import exclusive_scan
        assert text.dtype == torch.uint8 and text.is_contiguous()
        s = _hip.stream(d)
        tiles = int(_hip.lib().mr_text_tiles(n))
        counts = torch.empty(tiles, dtype=torch.int64, device=d)
        nls = torch.empty(tiles, dtype=torch.int64, device=d) if want_line else None
        _hip.call("mr_text_count", _hip.ptr(text), n, mode, byte, _hip.ptr(counts), _hip.ptr(nls), s)
        off, total = exclusive_scan(counts)
        loff = exclusive_scan(nls)[0] if want_line else None
        m = int(total.item())
        pos = torch.empty(m, dtype=torch.int64, device=d)
        ln = torch.empty(m, dtype=torch.int32, device=d) if want_len else None
        line = torch.empty(m, dtype=torch.int64, device=d) if want_line else None
        _hip.call("mr_text_emit", _hip.ptr(text), n, mode, byte, _hip.ptr(off), m, _hip.ptr(pos), _hip.ptr(ln),
                  _hip.ptr(loff), _hip.ptr(line), s)
        return pos, ln, line
    b = _np(text)
    if mode == 1:
        pos = np.flatnonzero(b == byte).astype(np.int64)
        ln = None
    else:
        ws = _WS_TABLE[b]
        d_ = np.diff((~ws).astype(np.int8), prepend=0, append=0)
        pos = np.flatnonzero(d_ == 1).astype(np.int64)
        ends = np.flatnonzero(d_ == -1).astype(np.int64)
        ln = torch.from_numpy((ends - pos).astype(np.int32))
    line = None
    if want_line:  # newlines strictly before each position
        line = torch.from_numpy(np.searchsorted(np.flatnonzero(b == 10), pos, side="left").astype(np.int64))
    return torch.from_numpy(pos), ln, line


def tokens(text: torch.Tensor, lines: bool = False):
    """(starts int64, lens int32) of every whitespace token (maximal run of
    bytes outside Lua's ``%s``), in text order; with ``lines=True`` also the
    0-based line number of each token (int64; = ``line_index(text, starts)``,
    from the same pass over the bytes)."""
    st, ln, line = _scan(text, 0, 0, True, lines)
    return (st, ln, line) if lines else (st, ln)


def ngrams(text: torch.Tensor, n: int = 2):
    """(starts int64, lens int32) of the n-gram starting at every whitespace
    token: the byte span from the token's start to the end of the (n-1)-th
    token after it on the same line (a newline ends an n-gram; other
    whitespace between the tokens is part of the span); lens 0 where fewer
    than n tokens are left on the line (``emit.spans`` skips those).  One
    pass over the bytes on the GPU (the token scan's kernel, spans from the
    tile's whitespace / newline masks)."""
    n = int(n)
    if not 1 <= n <= 64:
        raise ValueError("ngrams: 1 <= n <= 64")
    if n == 1:
        return tokens(text)
    if text.is_cuda and text.numel():
        st, ln, _ = _scan(text, 0, n, True)
        return st, ln
    st, ln, line = _scan(text, 0, 0, True, True)
    m = st.numel()
    out = torch.zeros(m, dtype=torch.int32)
    if m >= n:
        end = st[n - 1:] + ln[n - 1:].to(torch.int64)
        same = line[n - 1:] == line[:m - n + 1]
        out[:m - n + 1] = torch.where(same, end - st[:m - n + 1], torch.zeros_like(end)).to(torch.int32)
    return st, out


def find_byte(text: torch.Tensor, byte: int) -> torch.Tensor:
    """Positions (int64, ascending) of every byte equal to ``byte``."""
    return _scan(text, 1, int(byte) & 0xFF, False)[0]


def lines(text: torch.Tensor):
    """(starts int64, lens int32) of every line (bytes between newlines, the
    newline excluded; empty lines included; a final newline does not open an
    empty last line)."""
    n = text.numel()
    nl = find_byte(text, 10)
    d = text.device
    zero = torch.zeros(1, dtype=torch.int64, device=d)
    starts = torch.cat([zero, nl + 1])
    ends = torch.cat([nl, torch.full((1,), n, dtype=torch.int64, device=d)])
    if n == 0 or (nl.numel() and int(nl[-1]) == n - 1):
        starts, ends = starts[:-1], ends[:-1]
    return starts, (ends - starts).to(torch.int32)


def line_index(text: torch.Tensor, positions: torch.Tensor, newlines: torch.Tensor | None = None) -> torch.Tensor:
    """0-based line number of each byte position (int64)."""
    nl = find_byte(text, 10) if newlines is None else newlines
    return torch.searchsorted(nl, positions, right=False)


def field(text: torch.Tensor, starts: torch.Tensor, lens: torch.Tensor, sep: int | bytes, k: int):
    """Span of field ``k`` (0-based) of each line given by (starts, lens),
    fields separated by the byte ``sep``; a trailing ``\\r`` is dropped.  A
    missing field (also every field of an empty line) has start -1 and
    length 0."""
    if isinstance(sep, (bytes, str)):
        sep = (sep.encode() if isinstance(sep, str) else sep)[0]
    m = starts.numel()
    d = text.device
    if text.is_cuda:
        st = starts.to(torch.int64).contiguous()
        ln = lens.to(torch.int32).contiguous()
        fs = torch.empty(m, dtype=torch.int64, device=d)
        fl = torch.empty(m, dtype=torch.int32, device=d)
        _hip.call("mr_text_field", _hip.ptr(text), _hip.ptr(st), _hip.ptr(ln), m, int(sep), int(k), _hip.ptr(fs),
                  _hip.ptr(fl), _hip.stream(d))
        return fs, fl
    b = _np(text).tobytes()
    fs = np.full(m, -1, np.int64)
    fl = np.zeros(m, np.int32)
    sb = bytes([sep])
    for i, (s, n) in enumerate(zip(_np(starts).tolist(), _np(lens).tolist())):
        line = b[s:s + n] if n > 0 else b""
        if line.endswith(b"\r"):
            line = line[:-1]
        if not line:
            continue  # an empty line has no fields
        parts = line.split(sb)
        if k < len(parts):
            fs[i] = s + sum(len(p) + 1 for p in parts[:k])
            fl[i] = len(parts[k])
    return torch.from_numpy(fs), torch.from_numpy(fl)


def _parse_host(b: bytes, s: int, n: int, kind):
    if s < 0:
        raise ValueError
    tok = b[s:s + n].decode("ascii").strip(" \t\n\v\f\r")
    if not tok:
        raise ValueError
    if kind is int:
        if not (tok.lstrip("+-").isdigit()) or len(tok.lstrip("+-")) > 19:
            raise ValueError
        return int(tok)
    if any(c not in "0123456789+-.eE" for c in tok):
        raise ValueError
    return float(tok)


def _parse(text, starts, lens, kind, check: bool):
    m = starts.numel()
    d = text.device
    dt = torch.float64 if kind is float else torch.int64
    if text.is_cuda:
        st = starts.to(torch.int64).contiguous()
        ln = lens.to(torch.int32).contiguous()
        out = torch.empty(m, dtype=dt, device=d)
        err = torch.zeros(1, dtype=torch.int32, device=d)
        name = "mr_text_parse_f64" if kind is float else "mr_text_parse_i64"
        _hip.call(name, _hip.ptr(text), _hip.ptr(st), _hip.ptr(ln), m, _hip.ptr(out), _hip.ptr(err), _hip.stream(d))
        if check and int(err.item()):
            raise ValueError("malformed number in the parsed spans")
        return out
    b = _np(text).tobytes()
    out = np.zeros(m, np.float64 if kind is float else np.int64)
    bad = False
    for i, (s, n) in enumerate(zip(_np(starts).tolist(), _np(lens).tolist())):
        try:
            out[i] = _parse_host(b, s, n, kind)
        except (ValueError, UnicodeDecodeError):
            out[i] = np.nan if kind is float else 0
            bad = True
    if check and bad:
        raise ValueError("malformed number in the parsed spans")
    return torch.from_numpy(out)


def parse_f64(text: torch.Tensor, starts: torch.Tensor, lens: torch.Tensor, check: bool = False) -> torch.Tensor:
    """Decimal numbers of the spans as float64 (``[+-]digits[.digits][e[+-]digits]``
    with surrounding whitespace): correctly rounded when the significant
    digits fit 53 bits and the exponent is within +-22 (what Python's float()
    gives), a few ulp off otherwise.  Malformed spans give NaN (``check``:
    raise instead, one host synchronisation)."""
    return _parse(text, starts, lens, float, check)


def parse_i64(text: torch.Tensor, starts: torch.Tensor, lens: torch.Tensor, check: bool = False) -> torch.Tensor:
    """Decimal integers of the spans as int64 (malformed: 0, or raise with ``check``)."""
    return _parse(text, starts, lens, int, check)


def csv_rows(text: torch.Tensor, key: int = 0, values=(1,), sep: str | int = ","):
    """The rows of a CSV-like text as the general plane's ``emit.csv`` folds
    them: (key starts, key lens, [one tensor or the constant 1 per value
    input]) — key = field ``key`` of each line, input i = the number in field
    ``values[i]`` (None: the constant 1).  A row with a missing key or value
    field or a value that does not parse gets key length 0 (emit skips it).
    The specification of the fused kernel (csrc/hip/generic.hip mr_csv_fold)."""
    sep = sep if isinstance(sep, int) else ord(sep)
    ls, ll = lines(text)
    ks, kl = field(text, ls, ll, sep, key)
    ok = ks >= 0
    cols, cache = [], {}
    for v in values:
        if v is None:
            cols.append(1)
            continue
        if v not in cache:
            fs, fl = field(text, ls, ll, sep, v)
            x = parse_f64(text, fs, fl)
            ok &= (fs >= 0) & ~torch.isnan(x)
            cache[v] = x
        cols.append(cache[v])
    kl = torch.where(ok, kl, torch.zeros_like(kl))
    return ks, kl, cols
