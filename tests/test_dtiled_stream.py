"""The d-tiled kernel's LDS ring protocol on the CPU (csrc/fa_dtiled_stream.hpp).

fa_fwd_dt_kernel takes its wait counts, barrier positions, issue lead and slot arithmetic from
DtStream; tests/native/dtiled_stream_test.cpp replays that protocol, one wave's DMA pieces in
issue order under `s_waitcnt vmcnt(N)` semantics, for every (d, d_tile_qk, d_tile_v)
instantiation, the shipped 4-slot ring and the measured variants (3 / 5 / 8 slots, chunks in
pairs), at 1-9 tiles: no chunk is read before all its pieces landed, from a slot other than its
own, or overwritten before every wave passed the barrier after its last read.  (A wait count
one chunk too generous, or a slot off by one, fails it: checked by mutation when written.)
"""
import json
import os
import subprocess

from conftest import ROOT


def test_dtiled_ring_protocol(tmp_path):
    exe = tmp_path / "dtiled_stream_test"
    subprocess.run(["g++", "-O1", "-std=c++17", "-Wall", "-Werror", "-o", str(exe),
                    os.path.join(ROOT, "tests", "native", "dtiled_stream_test.cpp")], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    rows = [json.loads(x) for x in r.stdout.splitlines()]
    assert rows and all(x["ok"] for x in rows)
    tiles = {(x["dq"], x["dv"]) for x in rows}
    assert tiles == {(a, b) for a in (32, 64, 128) for b in (32, 64, 128)}
    shipped = [x for x in rows if x["slots"] == 4 and x["grp"] == 1 and x["tiles"] == 9]
    # (a paired-ring request at an odd number of chunks per tile falls back to one at a time)
    assert {(x["d"], x["dq"], x["dv"]) for x in shipped} == {(d, a, b) for d in (384, 512) for a in (32, 64, 128)
                                                             for b in (32, 64, 128)}
    # the shipped ring keeps chunks in flight at its steady waits (it does not drain each time)
    assert all(x["steady"] > 0 and x["max_inflight"] > 0 for x in shipped)
