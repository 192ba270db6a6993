"""lua_mapreduce_1_amd — an MI355X-native MapReduce engine.

Same public surface as the reference package (/root/reference/mapreduce/init.lua:19-40):
``{_VERSION, _NAME, worker, server, utils, tuple, persistent_table, utest}``,
plus the device data plane (``ops``), the SPMD/RCCL engine (``parallel``) and
workload families (``models``).
"""
from __future__ import annotations

_VERSION = "0.3.7"
_NAME = "mapreduce"

from . import utils  # noqa: E402
from .utils.tuple import tuple  # noqa: E402,A004
from .runtime.server import server  # noqa: E402
from .runtime.worker import worker  # noqa: E402
from .runtime.persistent_table import persistent_table  # noqa: E402


def utest(connection_string=None, dbname: str = "test") -> None:
    """Integrity test (init.lua:36-38 runs server.utest)."""
    from .runtime import server as _s
    _s.utest(connection_string, dbname)


def spmd(params: dict, **kw):
    """SPMD engine for a task table (server:configure's keys plus
    ``checkpoint_dir``): the HIP data plane when the map module has a
    ``device_mapfn`` (parallel/spmd.py), the reference's host semantics
    otherwise (parallel/spmd_host.py).  ``.run()`` iterates to completion."""
    from .runtime import modules
    if modules.field(modules.load(params["mapfn"]), "device_mapfn") is not None:
        from .parallel.spmd import SPMDEngine
        return SPMDEngine(params, **kw)
    from .parallel.spmd_host import HostSPMDEngine
    return HostSPMDEngine(params, **kw)


__all__ = ["_VERSION", "_NAME", "worker", "server", "utils", "tuple", "persistent_table", "utest", "spmd"]
