#!/bin/bash
# Fast A/B builds: libfa_mi355x.so with only the contiguous bf16 forward kernels of one head dim
# (fa_fwd.hip with -DFA_LITE_D=<d>) plus the C ABI -- seconds instead of minutes per variant.
#   bash scripts/build_lite.sh <d> name1 "FLAGS1" name2 "FLAGS2" ...
# -> exploring_flash_attention_amd/_lib/ab/<name>.so  (time them with scripts/ab.py)
set -e
cd "$(dirname "$0")/.."
D=$1; shift
CS=exploring_flash_attention_amd/csrc
OUT=exploring_flash_attention_amd/_lib/ab
mkdir -p $OUT /tmp/fa_lite
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -ffp-contract=fast -fno-slp-vectorize -mllvm --amdgpu-mfma-vgpr-form"
/opt/rocm/bin/hipcc $FL -x hip -c scripts/lite/fa_lite_stubs.cpp -o /tmp/fa_lite/stubs.o
pids=()
names=()
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  ( /opt/rocm/bin/hipcc $FL -DFA_LITE_D=$D $flags -x hip -c $CS/fa_fwd.hip -o /tmp/fa_lite/$name.o &&
    /opt/rocm/bin/hipcc $FL $flags -x hip -c $CS/fa_capi.cpp -o /tmp/fa_lite/$name.capi.o &&
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $OUT/$name.so /tmp/fa_lite/$name.o /tmp/fa_lite/$name.capi.o /tmp/fa_lite/stubs.o &&
    echo "built $name ($flags)" ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
