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


def test_gpus_request_beyond_the_node_fails_loudly():
    """`bench.py --gpus 2` with no launcher on a node with fewer GPUs (this container has none)
    exits non-zero with a message -- never a one-GPU line labelled n_gpus 1."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert r.stdout.strip() == "" and "--gpus 2 requested" in r.stderr


def test_world_size_disagreeing_with_gpus_is_an_error():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 2 and "disagree" in r.stderr and r.stdout.strip() == ""


def test_spawn_ranks_starts_n_ranks_and_propagates_failure(tmp_path):
    """The launcher bench.py uses for --gpus N: N processes with RANK / WORLD_SIZE set, and a
    failing rank makes the whole launch fail (non-zero status)."""
    sys.path.insert(0, ROOT)
    import bench
    script = tmp_path / "rank.py"
    script.write_text(
        "import os, sys\n"
        "r, w = os.environ['RANK'], os.environ['WORLD_SIZE']\n"
        "open(os.path.join(sys.argv[1], 'rank' + r), 'w').write(w)\n"
        "sys.exit(7 if sys.argv[2] == r else 0)\n")
    assert bench.spawn_ranks(3, str(script), [str(tmp_path), "-1"]) == 0
    assert sorted(p.name for p in tmp_path.glob("rank[0-9]")) == ["rank0", "rank1", "rank2"]
    assert all((tmp_path / f"rank{i}").read_text() == "3" for i in range(3))
    for p in tmp_path.glob("rank[0-9]"):
        p.unlink()
    assert bench.spawn_ranks(2, str(script), [str(tmp_path), "1"]) != 0


def test_extra_shapes_split_where_the_library_splits():
    """The split-KV bench extras: the two low-parallelism shapes are planned with more than one
    partial per query tile by the library (on the MI355X's 256 CUs), their `unsplit` twins
    with one."""
    sys.path.insert(0, ROOT)
    import bench
    from exploring_flash_attention_amd import ops
    shapes = {s[0]: s for s in bench.EXTRA_SHAPES}
    for base, ppt in (("b1h1_l16k", 4), ("b1h2_l4k", 4)):
        _, B, H, L, d, _, kvt, grp = shapes[base + "_splitkv"]
        assert grp is None and ops.v2_split_plan(B, H, L, d, kvt)[2] == ppt
        _, B, H, L, d, _, kvt, grp = shapes[base + "_unsplit"]
        blocks = ops.v2_split_plan(B, H, L, d, kvt)[0]
        assert grp == "all" and ops.v2_split_plan(B, H, L, d, kvt, blocks_per_workgroup=blocks)[2] == 1


def test_splitkv_scaling_field_at_mocked_two_ranks():
    """At N > 1 the C5 split-KV measurement (north_star's multi-GPU row) is a top-level field of
    the bench line, carrying ms, whole-job rate, frac and the exchange's own ms / GB/s."""
    sys.path.insert(0, ROOT)
    import bench
    c5 = {"ms": 15.0, "tflops": 2345.6, "frac": 0.469, "ranks": 2, "exchange": "pairwise send/recv",
          "breakdown_max_over_ranks": {"partial_ms": 14.1, "combine_ms": 0.4, "exchange_ms": 3.2,
                                       "exchange_gbps": 167.8, "exchange_bytes_per_rank": 537_000_000}}
    rec = bench.splitkv_scaling_field(c5, 2)
    assert rec["ranks"] == 2 and rec["ms"] == 15.0 and rec["frac"] == 0.469
    assert rec["value"] == 2345600.0 and rec["exchange_ms"] == 3.2 and rec["exchange_gbps"] == 167.8
    err = bench.splitkv_scaling_field({"error": "no result within 240 s", "ranks": 2}, 2)
    assert err["error"].startswith("no result") and "ms" not in err


def test_kernel_labels_come_from_the_library():
    """bench.py names the kernels the library reports having launched (fa_last_kernels through
    ops.launched_kernels), in call order without repeats -- no restated launch rule to drift
    from fa_fwd.hip."""
    import contextlib
    sys.path.insert(0, ROOT)
    import bench

    class FakeOps:
        @contextlib.contextmanager
        def launched_kernels(self):
            log = []
            self.log = log
            yield log

    ops = FakeOps()

    def step():  # a C5-like step: three partial chunks and a combine
        ops.log.extend(["fa_fwd16_kernel<partial, strided> [grid 256]"] * 3 + ["fa_combine_kernel [grid 64]"])
    assert bench.launched(ops, step) == "fa_fwd16_kernel<partial, strided> [grid 256] + fa_combine_kernel [grid 64]"
    assert bench.launched(ops, lambda: None) is None


def test_extra_traffic_records_are_labelled():
    """Every bench extra with a traffic entry reports measured bytes, the algorithmic bytes and
    the kernel the PMC pass measured."""
    import bench
    for name, B, H, L, d, *_ in bench.EXTRA_SHAPES:
        tr = bench.extra_traffic(name, B, H, L, d)
        if tr is None:
            continue
        assert tr["algorithmic_bytes"] == 8 * B * H * L * d
        assert tr["bytes_per_launch"] > 0 and tr["ratio"] > 0
        assert tr["kernel"] and tr["kernel"] != "(unlabelled)", name
