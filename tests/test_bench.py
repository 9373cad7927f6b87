"""bench.py's host-side logic on CPU: the C5 watchdog fails the run, the head sample, the
usable-core count."""
import os
import subprocess
import sys

from conftest import ROOT


def test_watchdog_exits_nonzero_and_prints_partial_line():
    code = (
        "import sys, time; sys.path.insert(0, %r); import bench\n"
        "bench.start_watchdog(0.3, 0, lambda: {'metric': 'm', 'extra': {'c5_splitkv_dist': {'error': 'hung'}}})\n"
        "time.sleep(30)\n" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 3, (r.returncode, r.stderr)
    assert '"error": "hung"' in r.stdout and "watchdog fired" in r.stderr


def test_watchdog_cancelled_is_silent():
    code = ("import sys, time; sys.path.insert(0, %r); import bench\n"
            "d = bench.start_watchdog(0.5, 1, lambda: None); d.cancel(); time.sleep(1.0)\n" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout == ""


def test_sample_heads_and_host_cores():
    sys.path.insert(0, ROOT)
    import bench
    hs = bench.sample_heads(32, 8)
    assert len(hs) == 16 and hs[0] == (0, 0) and hs[-1] == (31, 7)
    usable, total = bench.host_cores()
    assert 1 <= usable <= total == os.cpu_count()
    assert bench.cpu_model()
