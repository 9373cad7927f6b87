"""The chained d = 128 kernel's hand-counted vmcnt waits, checked in its gfx950 ISA (ADVICE
round 5): tests/native/chain_isa.hip instantiates fa_fwd16_chain_kernel (final and fused walk)
alone, hipcc compiles it to assembly here (no GPU needed, ~6 s), and scripts/check_vmcnt.py
requires the N youngest vector-memory operations in front of every hand-counted
`s_waitcnt vmcnt(N)` + `s_barrier` to be the ones allowed to stay in flight (the previous
item's O stores, the next item's Q^T loads, V(0) / K(1) in the prologue) -- never an LDS-DMA
piece the barrier must see landed."""
import os
import shutil
import subprocess
import sys

import pytest

from conftest import ROOT

HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-munsafe-fp-atomics", "-ffp-contract=fast",
         "-fno-slp-vectorize", "-mllvm", "--amdgpu-mfma-vgpr-form"]  # csrc/Makefile CXXFLAGS
sys.path.insert(0, os.path.join(ROOT, "scripts"))


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_chain_kernel_vmcnt_counts(tmp_path):
    import check_vmcnt
    mk = open(os.path.join(ROOT, "exploring_flash_attention_amd", "csrc", "Makefile")).read()
    for f in FLAGS:  # the flags the product is built with
        assert f.replace("gfx950", "$(ARCH)") in mk, f
    asm = tmp_path / "chain.s"
    subprocess.run([HIPCC, *FLAGS, "-x", "hip", "--cuda-device-only", "-S",
                    os.path.join(ROOT, "tests", "native", "chain_isa.hip"), "-o", str(asm)],
                   check=True, capture_output=True, text=True, timeout=600)
    bad, rows = check_vmcnt.check(str(asm))
    assert bad == 0, "\n".join(rows)
    kinds = " ".join(rows)
    # all three hand-counted kinds present (final mode) and the fused walk's EPI (20 stores)
    assert "EPI: ok" in kinds and "QNEXT: ok" in kinds and "prologue: ok" in kinds
    assert any("vmcnt(20)" in r and "EPI: ok" in r for r in rows)


def test_vmcnt_checker_catches_an_underwait(tmp_path):
    """A wait counting 8 stores with only 7 issued behind the DMA pieces (a piece in the 8
    youngest) is reported."""
    import check_vmcnt
    body = ["_ZN2fa21fa_fwd16_chain_kernelIDF16bLi0EEEvNS_7FwdArgsEi:"]
    body += ["\tbuffer_load_dwordx4 v1, s[0:3], 0 offen lds"] * 4
    body += ["\tbuffer_store_dwordx4 v[0:3], v4, s[8:11], 0 offen"] * 7
    body += ["\ts_waitcnt vmcnt(8)", "\ts_barrier", "\ts_endpgm"]
    p = tmp_path / "bad.s"
    p.write_text("\n".join(body) + "\n")
    bad, rows = check_vmcnt.check(str(p))
    assert bad == 1 and "VIOLATION" in rows[0]
