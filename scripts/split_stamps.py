"""Anatomy of the one-shot split-KV launch (fa_fwd16_kernel<fused>) from an FA_STAMPS=1 build:
where the small split shapes' time goes outside the KV loop.

    bash scripts/build_variants.sh stamps "-DFA_STAMPS=1"
    python scripts/split_stamps.py exploring_flash_attention_amd/_lib/ab/stamps.so [b1h2l4k|b1h1l16k]

Runs fa_fwd_v2 back to back (clock warm-up), then one stamped launch, and reports per workgroup
(wave 0, s_memtime cycles, converted with each XCD's own clock): prologue wait, first QK^T, KV
loop, hand-off (loop end -> verdict), the last workgroup's wait + combine + O retirement, and
on the 100 MHz realtime clock the launch's span from the first entry to the last end against
the HIP-event time of the same launch.  Diagnostic only: the stamps cost a few percent.
"""
import ctypes
import sys

import numpy as np
import torch

CFG = {"b1h2l4k": (1, 2, 4096, 128), "b1h1l16k": (1, 1, 16384, 128), "b1h4l4k": (1, 4, 4096, 128)}


def main():
    lib = ctypes.CDLL(sys.argv[1])
    B, H, L, d = CFG[sys.argv[2] if len(sys.argv) > 2 else "b1h2l4k"]
    lib.fa_fwd_v2_workspace_size.argtypes = [ctypes.c_int64] * 4 + [ctypes.c_int] * 3 + [
        ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_int)]
    lib.fa_fwd_v2.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int64] * 4 + [ctypes.c_int] * 3 + [
        ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    lib.fa_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    nb, ns = ctypes.c_size_t(), ctypes.c_int()
    assert lib.fa_fwd_v2_workspace_size(B, H, L, d, 4, 1, 4, ctypes.byref(nb), ctypes.byref(ns)) == 0
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn(B, H, L, d, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(3))
    o = torch.empty_like(q)
    ws = torch.zeros(nb.value, device="cuda", dtype=torch.uint8)
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def run():
        assert lib.fa_fwd_v2(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, L, d, 32, 32, 4,
                             ws.data_ptr(), nb.value, 1, 4, stream) == 0

    for _ in range(2000):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    run()
    e1.record()
    torch.cuda.synchronize()
    wall = e0.elapsed_time(e1) * 1e3
    buf = np.zeros(65536 * 16, dtype=np.uint64)
    assert lib.fa_debug_stamps(buf.ctypes.data, buf.nbytes) == 0
    s = buf.reshape(-1, 16).astype(np.int64)
    s = s[s[:, 0] != 0]
    nwg = len(s)
    xcc = s[:, 7] & 0xF
    rt0 = s[:, 8].min()
    ent, end = (s[:, 8] - rt0) * 0.01, (s[:, 9] - rt0) * 0.01  # us, one time base
    clk = (s[:, 5] - s[:, 0]) / np.maximum(end - ent, 1e-3)  # cycles per us, per workgroup
    xclk = {x: np.median(clk[xcc == x]) for x in np.unique(xcc)}
    cpu = np.array([xclk[x] for x in xcc])
    last = s[:, 12] == 1

    def us(a, b, m=None):
        dt = (s[:, b] - s[:, a]) / cpu
        return dt if m is None else dt[m]

    print(f"{sys.argv[2] if len(sys.argv) > 2 else 'b1h2l4k'}: B{B} H{H} L{L} d{d}, {nwg} workgroups "
          f"({last.sum()} tiles, {nwg // max(last.sum(), 1)} partials each); HIP events {wall:.1f} us; "
          f"realtime first entry -> last end {end.max():.1f} us; entries within {ent.max():.2f} us; "
          f"clock {np.median(cpu) / 1e3:.2f} GHz")
    rows = [("prologue wait", 0, 1, None), ("first QK^T", 1, 2, None), ("KV loop", 2, 3, None),
            ("loop end -> verdict (not last)", 3, 10, ~last), ("loop end -> verdict (last)", 3, 10, last),
            ("verdict -> combine start (last)", 10, 11, last), ("combine + O issue (last)", 11, 4, last),
            ("O retire (last)", 4, 5, last)]
    for nm, a, b, m in rows:
        dt = us(a, b, m)
        print(f"  {nm:34s} median {np.median(dt):6.2f}  p10 {np.percentile(dt, 10):6.2f}  "
              f"p90 {np.percentile(dt, 90):6.2f} us")
    life = us(0, 5)
    loop = us(2, 3)
    print(f"  lifetime median {np.median(life):.2f} us (last workgroups {np.median(life[last]):.2f}); KV loop "
          f"{np.median(loop):.2f} us = {np.median(loop) / np.median(life[last]):.0%} of a last workgroup's life")
    print(f"  realtime: last end {end.max():.1f} us, median end {np.median(end):.1f}, the last workgroups' ends "
          f"p10 {np.percentile(end[last], 10):.1f} / p90 {np.percentile(end[last], 90):.1f} us; launch overhead "
          f"outside the workgroups (HIP events - realtime span) {wall - end.max():.1f} us")


if __name__ == "__main__":
    main()
