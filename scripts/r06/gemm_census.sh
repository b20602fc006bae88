#!/bin/bash
# round-6: GEMM census of the current tree (every cmx_gemm call re-timed standalone, beside hipBLASLt)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 400 python3 -u scripts/gemm_census.py --out gpurun_out/r06/gemm_census.txt > gpurun_out/r06/gemm_census.log 2>&1
rc=$?; echo "census rc=$rc"; tail -5 gpurun_out/r06/gemm_census.log; exit $rc
