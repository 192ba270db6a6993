"""Host-side sanitizer runs of the native control plane.

The C++ coordinator (csrc/coord/coord.cpp, the MongoDB replacement) is built
together with a multi-threaded stress client (csrc/coord/coord_stress.cpp)
under ThreadSanitizer and under AddressSanitizer + UndefinedBehaviorSanitizer:
concurrent atomic job claims must hand every job out exactly once (the
reference's update-then-find claim could not guarantee that), persistent-table
locks must be exclusive, concurrent batched blob puts/gets/deletes must only
ever read intact bodies (they are swapped in whole outside the store lock),
long-poll claims must also hand every job out exactly once, and neither
sanitizer may report anything."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(ROOT, "csrc", "coord", "coord.cpp"), os.path.join(ROOT, "csrc", "coord", "coord_stress.cpp")]


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_coordinator_under_sanitizer(tmp_path, san):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no g++")
    exe = str(tmp_path / "coord_stress")
    r = subprocess.run([cxx, "-O1", "-g", "-std=c++17", "-pthread", f"-fsanitize={san}", "-fno-omit-frame-pointer",
                        "-fno-sanitize-recover=all", "-o", exe] + SRC, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66", ASAN_OPTIONS="detect_leaks=0")
    r = subprocess.run([exe, "8", "3000"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "coord_stress ok" in r.stdout
    assert "Sanitizer" not in r.stderr, r.stderr[-4000:]


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_split_loader_under_sanitizer(tmp_path, san):
    """The threaded split loader (csrc/host/loader.cpp) with 16 threads and
    4-16 KiB pieces, a consumer thread checking every job as soon as its
    ready flag is published, and a missing file: no sanitizer report."""
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no g++")
    exe = str(tmp_path / "loader_stress")
    src = [os.path.join(ROOT, "csrc", "host", "loader.cpp"), os.path.join(ROOT, "csrc", "host", "loader_stress.cpp")]
    r = subprocess.run([cxx, "-O1", "-g", "-std=c++17", "-pthread", f"-fsanitize={san}", "-fno-omit-frame-pointer",
                        "-fno-sanitize-recover=all", "-o", exe] + src, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66", ASAN_OPTIONS="detect_leaks=1")
    r = subprocess.run([exe, "48", "16", "3"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "loader_stress ok" in r.stdout
    assert "Sanitizer" not in r.stderr, r.stderr[-4000:]
