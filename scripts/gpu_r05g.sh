# round 5, call g: fused-mode chain A/B (C4 reference layout, C4 4 per wg, B1H1 L16k) + C3
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r05g
mkdir -p $O
export PYTHONPATH=$PWD
L=exploring_flash_attention_amd/_lib/ab
run() {  # name, args
  local n=$1; shift
  timeout -k 10 300 python -u scripts/ab.py --all "$@" $L/base.so $L/chain.so > $O/ab_$n.txt 2>&1 || { cat $O/ab_$n.txt; exit 1; }
  cat $O/ab_$n.txt
}
run c4g1 --config c4 --kvtpb 4 --bpw 1 --rounds 8
run c4g4 --config c4 --kvtpb 4 --bpw 4 --rounds 8
run b1h1 --shape 1,1,16384,128 --kvtpb 4 --rounds 12
run b2h2 --shape 2,2,16384,128 --kvtpb 4 --bpw 4 --rounds 12
run c3 --config c3 --rounds 12
