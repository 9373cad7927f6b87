#!/bin/bash
# Lite A/B builds of the d-tiled kernel: fa_fwd_dtiled.hip (+ the C ABI, a d=128 fa_fwd.hip and
# the stubs), one .so per flag set.   bash scripts/build_lite_dt.sh name1 "FLAGS1" name2 "FLAGS2" ...
set -e
cd "$(dirname "$0")/.."
CS=exploring_flash_attention_amd/csrc
OUT=exploring_flash_attention_amd/_lib/ab
mkdir -p $OUT /tmp/fa_lite
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -ffp-contract=fast -fno-slp-vectorize -mllvm --amdgpu-mfma-vgpr-form"
/opt/rocm/bin/hipcc $FL -x hip -c scripts/lite/fa_lite_stubs.cpp -o /tmp/fa_lite/stubs.o
/opt/rocm/bin/hipcc $FL -DFA_LITE_D=128 -x hip -c $CS/fa_fwd.hip -o /tmp/fa_lite/fwd128.o
/opt/rocm/bin/hipcc $FL -x hip -c $CS/fa_capi.cpp -o /tmp/fa_lite/capi.o
pids=()
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  src=$CS/fa_fwd_dtiled.hip; case $flags in *DT_OLD*) src=$CS/fa_fwd_dtiled_old.hip ;; esac
  # a flag set naming FA_DT_AGPR builds the d-tiled file without --amdgpu-mfma-vgpr-form
  FLD=$FL; case $flags in *FA_DT_AGPR*) FLD=${FL/ -mllvm --amdgpu-mfma-vgpr-form/} ;; esac
  ( /opt/rocm/bin/hipcc $FLD $flags -x hip -c $src -o /tmp/fa_lite/$name.dt.o &&
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $OUT/$name.so /tmp/fa_lite/$name.dt.o /tmp/fa_lite/fwd128.o \
        /tmp/fa_lite/capi.o /tmp/fa_lite/stubs.o && echo "built $name ($flags)" ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
