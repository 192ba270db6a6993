"""Worker -> GPU placement (utils/gpu_slots.py): lowest free lock-file slot,
device = slot % ndev, a dead worker's slot is reused."""
import subprocess
import sys
import time

from lua_mapreduce_1_amd.utils import gpu_slots
from lua_mapreduce_1_amd.runtime import worker as worker_mod


def test_slots_in_process(tmp_path):
    gpu_slots.utest()
    slots = [gpu_slots.claim(8, str(tmp_path)) for _ in range(10)]
    assert [s.device for s in slots] == [0, 1, 2, 3, 4, 5, 6, 7, 0, 1]
    for s in slots:
        s.release()


def test_slot_of_a_killed_worker_is_reused(tmp_path):
    code = ("import sys, time; sys.path.insert(0, sys.argv[1]);"
            "from lua_mapreduce_1_amd.utils import gpu_slots as g;"
            "s = g.claim(4, sys.argv[2]); print(s.slot, flush=True); time.sleep(60)")
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.Popen([sys.executable, "-c", code, root, str(tmp_path)], stdout=subprocess.PIPE, text=True)
    try:
        assert p.stdout.readline().strip() == "0"
        mine = gpu_slots.claim(4, str(tmp_path))
        assert (mine.slot, mine.device) == (1, 1)  # slot 0 is held by the other process
    finally:
        p.kill()
        p.wait()
    time.sleep(0.05)
    again = gpu_slots.claim(4, str(tmp_path))
    assert again.slot == 0  # SIGKILL released the lock
    again.release()
    mine.release()


def test_worker_gpu_option():
    w = worker_mod.worker.new(None, "gpu_slot_db")
    assert w.gpu == "auto"
    w.configure(gpu="none")
    assert gpu_slots.place_worker(w.gpu) is None
    assert gpu_slots.place_worker("auto") is None  # no GPU here / one GPU: torch's default device
