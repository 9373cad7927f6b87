#!/bin/bash
# Build A/B variants of libfa_mi355x.so into exploring_flash_attention_amd/_lib/ab/<name>.so
# usage: bash scripts/build_variants.sh name1 "FLAGS1" name2 "FLAGS2" ...
set -e
cd "$(dirname "$0")/../exploring_flash_attention_amd/csrc"
mkdir -p ../_lib/ab
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  make -s -j8 BUILD=build_ab/$name OUT=../_lib/ab/$name.so EXTRA="$flags" ../_lib/ab/$name.so >/dev/null
  echo "built $name ($flags)"
done
