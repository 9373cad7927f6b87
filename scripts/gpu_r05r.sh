# round 5, call r: d-tiled kernel at 32 query rows per wave (one workgroup per CU, O^T in AGPRs)
# against the shipped 16-row kernel, d = 384 / 512, bitwise compare
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r05r
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 500 bash scripts/ab_dtiled.sh dt_base dt_q2 > $O/ab_dt.txt 2>&1
rc=$?; cat $O/ab_dt.txt; exit $rc
