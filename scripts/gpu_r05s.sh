# round 5, call s: timing probe of the 32-row d-tiled kernel WITHOUT the O rescale (wrong outputs by design): the ceiling of a rescale-free 32-row kernel
# against the shipped 16-row kernel, d = 384 / 512, bitwise compare
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r05s
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 500 bash scripts/ab_dtiled.sh dt_base dt_q2nr > $O/ab_dt.txt 2>&1
rc=$?; cat $O/ab_dt.txt; exit $rc
