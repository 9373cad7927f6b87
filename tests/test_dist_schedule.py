"""The multi-GPU split-KV exchange schedule on the CPU.

fa_fwd_v2_dist's schedule -- which chunk each step sends where, which rank it receives from,
the own chunk's path, and the communicator latch after a part-way failure -- lives in
exploring_flash_attention_amd/csrc/fa_dist_schedule.hpp with no HIP or RCCL in it.
tests/native/dist_schedule_test.cpp runs it for W = 1, 2, 3, 4, 8 in-process ranks over a
fake transport that moves the bytes (per-pair FIFO matching, as RCCL point-to-point orders
them; every step checked to be a perfect matching) and injects failures at every operation.
"""
import json
import os
import subprocess

from conftest import ROOT


def test_exchange_schedule_with_fake_transport(tmp_path):
    exe = tmp_path / "dist_schedule_test"
    subprocess.run(["g++", "-O1", "-std=c++17", "-Wall", "-Werror", "-o", str(exe),
                    os.path.join(ROOT, "tests", "native", "dist_schedule_test.cpp")], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    rows = [json.loads(x) for x in r.stdout.splitlines()]
    ex = [x for x in rows if x["case"] == "exchange"]
    assert {(x["world"], x["pipelined"]) for x in ex} == {(w, p) for w in (1, 2, 3, 4, 8) for p in (0, 1)}
    assert all(x["ok"] and x["steps_posted"] == x["world"] * (x["world"] - 1) for x in ex)
    fails = [x for x in rows if x["case"] == "failure"]
    assert all(x["ok"] and x["status"] != 0 for x in fails)
    # a failure after step 1 was posted leaves the communicator broken
    late = [x for x in fails if x["op"] in ("fence_to_exchange", "post_step", "partial_chunk") and x["step"] > 1]
    assert late and all(x["broken"] for x in late)
    assert any(not x["broken"] for x in fails if x["step"] == 1)
