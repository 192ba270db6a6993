"""User-module loading (the reference's ``require`` of module names).

Module names accept ``/`` or ``.`` separators and an optional ``.py``/``.lua``
suffix (execute_server.lua:37-39 ``normalize``).  A module may also be given
directly as a Python module object, a class/instance, or a dict with the
function fields.  ``init(args)`` runs once per distinct init function
(job.lua:64-73).  Note: the reference passes an undefined global to the
map/reduce modules' ``init`` (job.lua:369); here every
``init`` receives ``init_args``.
"""
from __future__ import annotations

import importlib
import types
from typing import Any

_modules: dict[str, Any] = {}
_initialized: set[int] = set()


def normalize(name: str) -> str:
    n = name.replace("/", ".")
    for suf in (".py", ".lua"):
        if n.endswith(suf):
            n = n[: -len(suf)]
    return n


class _DictModule(types.SimpleNamespace):
    pass


def load(name_or_obj) -> Any:
    if name_or_obj is None:
        return None
    if isinstance(name_or_obj, str):
        n = normalize(name_or_obj)
        m = _modules.get(n)
        if m is None:
            m = importlib.import_module(n)
            _modules[n] = m
        return m
    if isinstance(name_or_obj, dict):
        return _DictModule(**name_or_obj)
    return name_or_obj


def field(mod, name: str, default=None):
    if mod is None:
        return default
    if isinstance(mod, dict):
        return mod.get(name, default)
    v = getattr(mod, name, default)
    # a package whose function name equals a submodule name (WordCount.taskfn
    # both as function of the single-module form and as split module): once
    # the submodule is imported the attribute is the module -> use its field.
    if isinstance(v, types.ModuleType):
        v = getattr(v, name, default)
    return v


def init_once(mod, args, seen: set | None = None) -> None:
    """Call the module's ``init(args)`` unless this init function already ran
    (in ``seen``: one task's dedup set, job.lua:64-73; default: the process-wide
    set, reset between tasks by :func:`reset`)."""
    f = field(mod, "init")
    if f is None:
        return
    seen = _initialized if seen is None else seen
    key = id(f)
    if key in seen:
        return
    f(args)
    seen.add(key)


def reset() -> None:
    """Forget initialisations (job.reset_cache analogue between tasks)."""
    _initialized.clear()


def name_of(name_or_obj) -> str | None:
    """Serializable module reference stored in the task document."""
    if name_or_obj is None:
        return None
    if isinstance(name_or_obj, str):
        return normalize(name_or_obj)
    if isinstance(name_or_obj, types.ModuleType):
        return name_or_obj.__name__
    raise TypeError("modules shared through the coordinator must be importable module names")
