"""Coordinator long polls (a blocking claim instead of
sleep-polling): JOB_CLAIM_WAIT holds a claim until a job can be claimed,
the task document changes, or the wait expires; WAIT_CHANGE returns once the
database has changed since a given mutation count; housekeeping ops that
change nothing (expire/fail/error-take with nothing to do) wake nobody."""
import threading
import time

from lua_mapreduce_1_amd.runtime import coordinator
from lua_mapreduce_1_amd.runtime.cnn import cnn
from lua_mapreduce_1_amd.runtime.task import task


def _later(dt, fn):
    t = threading.Thread(target=lambda: (time.sleep(dt), fn()))
    t.start()
    return t


def test_claim_wait_wakes_on_insert():
    cs = coordinator.start_local()
    a, b = cnn(cs, "lp1"), cnn(cs, "lp1")
    t0 = time.time()
    assert a.jobs("map_jobs").claim("w", "t", 0.0, wait=0.1) is None  # nothing: the full wait
    assert 0.09 <= time.time() - t0 < 1.0
    th = _later(0.05, lambda: b.jobs("map_jobs").insert({"_id": "1", "value": {"split": 0}}))
    t0 = time.time()
    j = a.jobs("map_jobs").claim("w", "t", 0.0, wait=5.0)
    dt = time.time() - t0
    th.join()
    assert j is not None and j["_id"] == "1" and dt < 1.0
    # claimed: a second long poll finds nothing
    assert a.jobs("map_jobs").claim("w", "t", 0.0, wait=0.05) is None


def test_claim_wait_ends_on_task_change():
    cs = coordinator.start_local()
    a, b = cnn(cs, "lp2"), cnn(cs, "lp2")
    th = _later(0.05, lambda: task(b).insert({"status": "REDUCE"}))
    t0 = time.time()
    assert a.jobs("map_jobs").claim("w", "t", 0.0, wait=5.0) is None
    th.join()
    assert time.time() - t0 < 1.0  # the worker goes back to re-read the task


def test_wait_change_and_quiet_housekeeping():
    cs = coordinator.start_local()
    a, b = cnn(cs, "lp3"), cnn(cs, "lp3")
    tk = task(a)
    tk.update()
    v = tk.version
    assert v >= 0
    # the server's monitor ops with nothing to do change nothing
    jb = b.jobs("map_jobs")
    jb.fail_broken(3)
    jb.expire(time.time(), 120.0)
    b.get_errors()
    t0 = time.time()
    assert a.wait_change(v, 0.1) == v and time.time() - t0 >= 0.09
    th = _later(0.05, lambda: b.insert_error("w", "boom"))
    t0 = time.time()
    v2 = a.wait_change(v, 5.0)
    th.join()
    assert v2 > v and time.time() - t0 < 1.0
    assert a.wait_change(-1, 0) == v2  # -1: the current count, no wait
