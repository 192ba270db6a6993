"""The tunables dataclass: defaults, typed env overrides,
and every knob documented with its MR_* variable."""
import dataclasses

from lua_mapreduce_1_amd.utils.config import Tunables


def test_defaults_and_overrides():
    t = Tunables.from_env({})
    assert t.default_sleep == 1.0 and t.force_shuffle is False and t.pipeline is True
    assert t.sort_rounds == 24 and t.map_sparsity == 8 and t.map_sparse_min_mb == 128.0
    s = Tunables.from_env({"MR_SORT_ROUNDS": "16", "MR_MAP_SPARSITY": "32", "MR_MAP_SPARSE_MIN_MB": "0"})
    assert s.sort_rounds == 16 and s.map_sparsity == 32 and s.map_sparse_min_mb == 0.0
    o = Tunables.from_env({"MR_DEFAULT_SLEEP": "0.05", "MR_FORCE_SHUFFLE": "1", "MR_PIPELINE": "0",
                           "MR_ROCTX": "1", "MR_SPIN_US": "0"})
    assert o.default_sleep == 0.05 and o.force_shuffle is True and o.pipeline is False
    assert o.roctx is True and o.spin_us == 0.0


def test_every_knob_documented():
    envs = [f.metadata["env"] for f in dataclasses.fields(Tunables)]
    assert len(envs) == len(set(envs)) and all(e.startswith("MR_") for e in envs)
    text = Tunables.from_env({}).describe()
    assert all(e in text for e in envs)
