"""The multi-GPU split-KV exchange's device operations on the CPU.

fa_fwd_v2_dist (exploring_flash_attention_amd/csrc/fa_dist.cpp) runs fa_dist_schedule.hpp's
schedule through fa_dist_ops.hpp's ExchangeOps: which partial kernel writes which workspace
bytes, which stream records / waits for which event, what each RCCL send and receive moves
and to which peer.  tests/native/dist_ops_test.cpp instantiates that same ExchangeOps over a
simulated node (in-order streams, HIP event semantics, per-pair point-to-point FIFOs, fake
partial kernels that check their arguments and write bytes naming producer / chunk / call) for
W = 1, 2, 3, 4, 8, four (dtype, partial dtype) pairs and several scheduling policies, two calls
back to back per case.

The mutation test edits fa_dist_ops.hpp -- offsets, sizes, peers, streams, strides, event
indices -- and requires the simulation to reject every edit that is a bug, and to accept the
edits that are not (an event index: a HIP wait binds to the event's latest record when it is
enqueued, so the per-step events are interchangeable -- the model must not flag them).
The reference has no multi-GPU code; the combine this exchange distributes is
flash_attention_v2/CUDA/flash_attention_v2.h:356-435.
"""
import json
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

TEST = os.path.join(ROOT, "tests", "native", "dist_ops_test.cpp")
OPS = os.path.join(ROOT, "exploring_flash_attention_amd", "csrc", "fa_dist_ops.hpp")


def _build(tmp_path, header=None, name="dist_ops_test"):
    exe = tmp_path / name
    cmd = ["g++", "-O1", "-std=c++17", "-Wall", "-Werror", "-o", str(exe), TEST]
    if header:
        cmd.insert(1, f'-DFA_DIST_OPS_HEADER="{header}"')
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def test_exchange_ops_on_simulated_ranks(tmp_path):
    exe = _build(tmp_path)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    rows = [json.loads(x) for x in r.stdout.splitlines()]
    ops = [x for x in rows if x["case"] == "ops"]
    assert {x["world"] for x in ops} == {1, 2, 3, 4, 8}
    assert {(x["dtype"], x["partial"]) for x in ops} == {("bf16", "fp16_scaled"), ("bf16", "fp32"),
                                                         ("fp16", "fp16"), ("fp64", "fp64")}
    # both exchange paths: pipelined (bf16 / fp16) and one launch + own-chunk copy (fp64)
    assert {x["pipelined"] for x in ops if x["world"] > 1} == {0, 1}
    assert all(x["ok"] for x in ops)
    fails = [x for x in rows if x["case"] == "failure"]
    assert fails and all(x["ok"] and x["status"] != 0 for x in fails)
    assert any(x["broken"] for x in fails) and any(not x["broken"] for x in fails)


# (what, original text in fa_dist_ops.hpp, replacement, the simulation must reject it)
MUTATIONS = [
    ("q row-view offset by the partial's element size",
     "(size_t)p * Lc * d * esize(dtype)", "(size_t)p * Lc * d * esize(pdtype)", True),
    ("q row-view offset off by one chunk",
     "(size_t)p * Lc * d * esize(dtype)", "(size_t)(p + 1) % (L / Lc) * Lc * d * esize(dtype)", True),
    ("q strides of the row view", "{H * L * d, L * d, d}", "{H * Lc * d, Lc * d, d}", True),
    ("chunk launch over all keys", "B, H, Lc, Lc, d, Lc, qst", "B, H, Lc, L, d, Lc, qst", True),
    ("one-launch chunk rows", "B, H, L, Lc, d, Lc, dtype", "B, H, L, Lc, d, L, dtype", True),
    ("fence: record on the exchange stream", "api.record(ev[e], s)", "api.record(ev[e], xs)", True),
    ("fence: the compute stream waits", "api.wait(xs, ev[e])", "api.wait(s, ev[e])", True),
    ("done: record on the compute stream", "api.record(ev[0], xs)", "api.record(ev[0], s)", True),
    ("done: the exchange stream waits", "api.wait(s, ev[0])", "api.wait(xs, ev[0])", True),
    ("fence event past the rank's events", "api.record(ev[e], s)", "api.record(ev[e + 1], s)", True),
    ("O chunk bytes by the input dtype",
     "const size_t chunk_o = (size_t)B * H * Lc * d * esize(pdtype);",
     "const size_t chunk_o = (size_t)B * H * Lc * d * esize(dtype);", True),
    ("lse chunk bytes without the scale exponent",
     "const size_t chunk_l = (size_t)B * H * Lc * lsize(dtype, pdtype);",
     "const size_t chunk_l = (size_t)B * H * Lc * 4;", True),
    ("O send to the source rank", "api.send(ws + so, chunk_o, dst, xs)", "api.send(ws + so, chunk_o, src, xs)", True),
    ("O receive from the destination rank", "api.recv(ws + ro, chunk_o, src, xs)",
     "api.recv(ws + ro, chunk_o, dst, xs)", True),
    ("lse send from the O buffer", "api.send(ws + sl, chunk_l, dst, xs)", "api.send(ws + so, chunk_l, dst, xs)", True),
    ("lse receive into the O slot", "api.recv(ws + rl, chunk_l, src, xs)", "api.recv(ws + ro, chunk_l, src, xs)",
     True),
    ("send on the compute stream", "api.send(ws + so, chunk_o, dst, xs)", "api.send(ws + so, chunk_o, dst, s)", True),
    ("group left open on success", "return api.group_end(e, st, dst, src);",
     "if (e) return api.group_end(e, st, dst, src);\n        return 0;", True),
    ("own-chunk copy reversed", "api.copy(ws + dst_off, ws + src_off, bytes, s)",
     "api.copy(ws + src_off, ws + dst_off, bytes, s)", True),
    ("receive lse region overlaps the send lse", "w.recv_o = w.send_lse + w.lse_bytes;",
     "w.recv_o = w.send_lse;", True),
    ("plan chunk bytes by the input dtype", "p.chunk_o = (size_t)BH * Lc * d * esize(pdtype);",
     "p.chunk_o = (size_t)BH * Lc * d * esize(dtype);", True),
    # not bugs: the model must accept them
    ("fence on event 0 (a wait binds to the latest record)", "api.record(ev[e], s)) return st;\n        return api.wait(xs, ev[e]);",
     "api.record(ev[0], s)) return st;\n        return api.wait(xs, ev[0]);", False),
    ("own-chunk copy on the exchange stream", "api.copy(ws + dst_off, ws + src_off, bytes, s)",
     "api.copy(ws + dst_off, ws + src_off, bytes, xs)", False),
]


@pytest.mark.parametrize("what,old,new,bug", MUTATIONS, ids=[m[0] for m in MUTATIONS])
def test_exchange_ops_mutations(tmp_path, what, old, new, bug):
    text = open(OPS).read()
    assert text.count(old) == 1, f"mutation anchor not unique in fa_dist_ops.hpp: {old!r}"
    # the mutated copy keeps the header's relative includes
    csrc = tmp_path / "exploring_flash_attention_amd" / "csrc"
    csrc.mkdir(parents=True)
    (tmp_path / "include").mkdir()
    for h in ("fa_mi355x.h", "fa_mi355x_dist.h"):
        shutil.copy(os.path.join(ROOT, "include", h), tmp_path / "include" / h)
    shutil.copy(os.path.join(os.path.dirname(OPS), "fa_dist_schedule.hpp"), csrc / "fa_dist_schedule.hpp")
    (csrc / "fa_dist_ops.hpp").write_text(text.replace(old, new))
    exe = _build(tmp_path, str(csrc / "fa_dist_ops.hpp"))
    r = subprocess.run([str(exe), "--quick"], capture_output=True, text=True, timeout=120)
    if bug:
        assert r.returncode != 0, f"simulation accepted the mutation: {what}"
    else:
        assert r.returncode == 0, f"simulation rejected a correct variant ({what}): {r.stderr}"
