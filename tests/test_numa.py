"""utils/numa.py: GPU -> NUMA node -> CPU mask, against a fake sysfs tree."""
import os

from lua_mapreduce_1_amd.utils import numa


def _fake_sys(tmp_path, pci="0000:c1:00.0", node=1, cpulist="0-3,8"):
    d = tmp_path / "bus" / "pci" / "devices" / pci
    d.mkdir(parents=True)
    (d / "numa_node").write_text(f"{node}\n")
    n = tmp_path / "devices" / "system" / "node" / f"node{node}"
    n.mkdir(parents=True)
    (n / "cpulist").write_text(cpulist + "\n")
    return str(tmp_path)


def test_parse_cpulist():
    assert numa.parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert numa.parse_cpulist("") == set()


def test_node_lookup_and_bind(tmp_path):
    allowed = sorted(os.sched_getaffinity(0))
    root = _fake_sys(tmp_path, cpulist=",".join(str(c) for c in allowed[:1]))
    assert numa.numa_node_of("0000:c1:00.0", root) == 1
    assert numa.numa_node_of("0000:ff:00.0", root) is None
    before = os.sched_getaffinity(0)
    try:
        got = numa.bind_cpus_to_node(1, root)
        assert got == {allowed[0]} and os.sched_getaffinity(0) == {allowed[0]}
    finally:
        os.sched_setaffinity(0, before)


def test_no_change_without_a_usable_node(tmp_path):
    root = _fake_sys(tmp_path, node=0, cpulist="100000")  # no allowed CPU on that node
    before = os.sched_getaffinity(0)
    assert numa.bind_cpus_to_node(0, root) is None
    assert numa.bind_cpus_to_node(None, root) is None
    assert os.sched_getaffinity(0) == before


def test_bind_to_gpu_without_gpu():
    info = numa.bind_to_gpu(0)
    assert info["cpus"] == 0 or info["node"] is not None
