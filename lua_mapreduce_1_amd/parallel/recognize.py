"""Recognise a host reducer that is a plain fold, so it runs batched on the device.

The reference's default contract is a per-key Lua ``reducefn(key, values,
emit)`` (/root/reference/mapreduce/job.lua:98-112,264-284); its WordCount
``reducefn2`` (examples/WordCount/reducefn2.lua, run by test.sh:37-53) is
``emit(sum(values))`` with no reducer flags and no batched form.  Here such a
module would take Python per key over every downloaded list (about 1 s per
step on the benchmark corpus, profiles/r4/general/wc_general.log).  When the
function's source is, exactly, one of

* ``emit(sum(values))`` / ``emit(min(values))`` / ``emit(max(values))``
  (the builtins, not shadowed in the function's globals), or
* ``acc = 0`` ; ``for v in values: acc += v`` (or ``acc = acc + v`` /
  ``acc = v + acc``) ; ``emit(acc)``

(docstrings and ``pass`` aside), the general plane runs the same fold over
every key's list at once (ops/segments.py) — the list semantics stay (the
reducer sees each key's whole list, the combiner still replaces the lists) and
only the execution moves.  Anything else, including any other statement, a
keyword argument or a default, is not recognised and keeps the host path.

Exactness: min / max always; ``sum`` only over int64 values (a float sum's
result depends on the order of additions, which the device does not keep).
Python's ``sum`` of int64 values is unbounded while the device's wraps at
2^63 — sums that large are out of the reference's range too (Lua numbers are
doubles).  ``Tunables.recognize_reducers`` (``MR_RECOGNIZE_REDUCERS=0``)
turns recognition off.
"""
from __future__ import annotations

import ast
import builtins
import inspect
import textwrap

FOLDS = ("sum", "min", "max")


def _body(fn):
    """The function's AST node, or None (no source: builtins, lambdas
    defined inline with others on one line, C functions...)."""
    try:
        src = textwrap.dedent(inspect.getsource(fn))
        tree = ast.parse(src)
    except (OSError, TypeError, SyntaxError, IndentationError):
        return None
    if len(tree.body) != 1 or not isinstance(tree.body[0], ast.FunctionDef):
        return None
    return tree.body[0]


def _plain_args(node) -> list[str] | None:
    a = node.args
    if a.posonlyargs or a.vararg or a.kwonlyargs or a.kwarg or a.defaults or node.decorator_list:
        return None
    if len(a.args) != 3:
        return None
    return [x.arg for x in a.args]


def _statements(node):
    body = list(node.body)
    if body and isinstance(body[0], ast.Expr) and isinstance(body[0].value, ast.Constant) \
            and isinstance(body[0].value.value, str):
        body = body[1:]  # the docstring
    return [s for s in body if not isinstance(s, ast.Pass)]


def _is_name(n, name: str) -> bool:
    return isinstance(n, ast.Name) and n.id == name


def _emit_of(stmt, emit: str):
    """The single positional argument of ``emit(<arg>)``, or None."""
    if not isinstance(stmt, ast.Expr) or not isinstance(stmt.value, ast.Call):
        return None
    c = stmt.value
    if not _is_name(c.func, emit) or c.keywords or len(c.args) != 1:
        return None
    return c.args[0]


def _builtin_fold(arg, values: str, fn) -> str | None:
    if not isinstance(arg, ast.Call) or not isinstance(arg.func, ast.Name) or arg.keywords or len(arg.args) != 1:
        return None
    name = arg.func.id
    if name not in FOLDS or not _is_name(arg.args[0], values):
        return None
    g = fn.__globals__
    b = g.get("__builtins__", builtins)
    b = b if isinstance(b, dict) else vars(b)
    if name in g or name in fn.__code__.co_freevars or b.get(name) is not getattr(builtins, name):
        return None  # shadowed: not the builtin
    return name


def _loop_sum(stmts, values: str, emit: str) -> bool:
    if len(stmts) != 3:
        return False
    init, loop, out = stmts
    if not (isinstance(init, ast.Assign) and len(init.targets) == 1 and isinstance(init.targets[0], ast.Name)
            and isinstance(init.value, ast.Constant) and init.value.value == 0
            and type(init.value.value) is int):
        return False
    acc = init.targets[0].id
    if not (isinstance(loop, ast.For) and isinstance(loop.target, ast.Name) and _is_name(loop.iter, values)
            and not loop.orelse and len(loop.body) == 1):
        return False
    v = loop.target.id
    if v in (acc, values, emit) or acc in (values, emit):
        return False
    s = loop.body[0]
    ok = False
    if isinstance(s, ast.AugAssign) and _is_name(s.target, acc) and isinstance(s.op, ast.Add) and _is_name(s.value, v):
        ok = True
    elif isinstance(s, ast.Assign) and len(s.targets) == 1 and _is_name(s.targets[0], acc) \
            and isinstance(s.value, ast.BinOp) and isinstance(s.value.op, ast.Add):
        lhs, rhs = s.value.left, s.value.right
        ok = (_is_name(lhs, acc) and _is_name(rhs, v)) or (_is_name(lhs, v) and _is_name(rhs, acc))
    return ok and _is_name(_emit_of(out, emit), acc)


def recognize(fn) -> str | None:
    """'sum' | 'min' | 'max' when ``fn(key, values, emit)`` is exactly that
    fold of its values (module docstring), else None."""
    if fn is None or not inspect.isfunction(fn):
        return None
    node = _body(fn)
    if node is None:
        return None
    args = _plain_args(node)
    if args is None:
        return None
    _, values, emit = args
    stmts = _statements(node)
    if len(stmts) == 1:
        arg = _emit_of(stmts[0], emit)
        return _builtin_fold(arg, values, fn) if arg is not None else None
    return "sum" if _loop_sum(stmts, values, emit) else None


def device_fold(op: str, dtype: str):
    """The batched device form of a recognised fold over lists of ``dtype``
    ('i64' | 'f64'), or None when it would not be exact (a float sum)."""
    from ..ops import segments as S
    if op == "sum" and dtype != "i64":
        return None
    f = {"sum": S.sum, "min": S.min, "max": S.max}[op]

    def fold(keys, off, val):
        return f(off, val)
    fold.__name__ = f"recognized_{op}"
    fold.recognized = op
    return fold
