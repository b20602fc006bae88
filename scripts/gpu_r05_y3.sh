#!/bin/bash
# streaming GEMM grid, stores in flight across the next step: GEMM tests + census A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r05_y3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r05_y3.log; grep -E "^FAILED" gpurun_out/pytest_r05_y3.log | head -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/gemm_census.py --ab GEMM_STREAM=0,1024 > gpurun_out/census_r05_y3.txt 2>&1 || exit 1
grep -v "Warning\|capture_end\|amdgpu.ids" gpurun_out/census_r05_y3.txt | head -14
