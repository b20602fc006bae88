#!/bin/bash
# Two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE: they do not fit one pass) over a short
# bench run, kernels filtered by regex, then the per-launch HBM-byte summary tagged with the
# bench workload (roofline.py reuses it only for the same workload).
#   scripts/pmc_pass.sh TAG "CMX-B2 train step 480x640 bs=2 K=40" gemm_grouped [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r02}
WORKLOAD=${2:-"CMX-B2 train step 480x640 bs=2 K=40"}
RE=${3:-gemm_grouped}
shift 3
mkdir -p gpurun_out
for C in FETCH_SIZE WRITE_SIZE; do
  CMX_BENCH_NO_ROOFLINE=1 timeout -k 10 240 rocprofv3 --pmc $C --kernel-include-regex "$RE" -d gpurun_out/pmc_${TAG}_$C -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/pmc_${TAG}_$C.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 scripts/pmc_summary.py gpurun_out/pmc_${TAG}.json $(ls gpurun_out/pmc_${TAG}_FETCH_SIZE/*/*.db gpurun_out/pmc_${TAG}_FETCH_SIZE/*.db 2>/dev/null | head -1) $(ls gpurun_out/pmc_${TAG}_WRITE_SIZE/*/*.db gpurun_out/pmc_${TAG}_WRITE_SIZE/*.db 2>/dev/null | head -1) "$WORKLOAD"
