"""Static checks of the inline-asm MFMA kernel (csrc/fa_fwd_w64.hip) in its compiled ISA.

Every MFMA there is inline asm, so the compiler's hazard recognizer does not see it.  This
compiles the file to assembly (hipcc -S, gfx950) and checks, for each kernel:
  1. the compiler never touches an AGPR outside our asm (a[0:255] are asm-owned);
  2. no VALU instruction reads or writes an MFMA's VGPR result while that MFMA may still
     be in flight (before an s_nop fence or 4 younger MFMAs);
  3. no VALU write of an MFMA source VGPR within the 2 wait states before the MFMA.
Exit status 1 on any finding.

    python scripts/check_asm_mfma.py [extra hipcc flags...]
"""
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "..", "exploring_flash_attention_amd", "csrc", "fa_fwd_w64.hip")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=fast",
         "-fno-slp-vectorize", "-mllvm", "--amdgpu-mfma-vgpr-form", "-x", "hip", "-S",
         "--cuda-device-only"]


def vregs(tok):
    out = set()
    for m in re.finditer(r"\bv\[(\d+):(\d+)\]", tok):
        out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
    for m in re.finditer(r"\bv(\d+)\b", tok):
        out.add(int(m.group(1)))
    return out


def check(body):
    issues = []
    inasm = False
    lines = []
    for raw in body.split("\n"):
        if "ASMSTART" in raw:
            inasm = True
            continue
        if "ASMEND" in raw:
            inasm = False
            continue
        t = raw.strip()
        if not t or t.startswith(";") or t.startswith(".") or t.endswith(":"):
            continue
        if not inasm and re.search(r"\ba\d+\b|a\[\d", t):
            issues.append(f"compiler AGPR use: {t}")
        lines.append(t)
    pending, mcount = {}, 0  # VGPR -> MFMA count at write
    for i, t in enumerate(lines):
        if t.startswith("s_nop 7"):
            pending.clear()
            continue
        if t.startswith("v_mfma"):
            mcount += 1
            pending = {r: c for r, c in pending.items() if mcount - c < 4}
            ops = t.split(None, 1)[1].split(",")
            if "v[" in ops[0]:
                for r in vregs(ops[0]):
                    pending[r] = mcount
            srcs = vregs(",".join(ops[1:3]))
            ws, j = 0, i - 1
            while j >= 0 and ws < 2:
                u = lines[j]
                if u.startswith("s_nop"):
                    ws += int(u.split()[1]) + 1
                elif u.startswith("v_") and not u.startswith("v_mfma") and " " in u:
                    if vregs(u.split(None, 1)[1].split(",")[0]) & srcs:
                        issues.append(f"VALU->MFMA ({ws} wait states): {u} | {t}")
                    ws += 1
                else:
                    ws += 1
                j -= 1
            continue
        if t.startswith("s_"):
            continue
        hit = vregs(t) & set(pending)
        if hit:
            issues.append(f"MFMA result read/written early: {t}")
    return issues


def main():
    out = "/tmp/fa_fwd_w64_check.s"
    subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *sys.argv[1:], SRC, "-o", out], check=True,
                   stderr=subprocess.DEVNULL)
    s = open(out).read()
    bad = 0
    for m in re.finditer(r"^(_ZN2fa17fa_fwd_w64_kernel\w+):(.*?)^\.Lfunc_end", s, re.S | re.M):
        issues = check(m.group(2))
        print(f"{m.group(1)}: {len(issues)} finding(s)")
        for x in issues[:10]:
            print("   ", x)
        bad += len(issues)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
