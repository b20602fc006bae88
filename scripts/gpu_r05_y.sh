#!/bin/bash
# streaming 64 x 64 GEMM grid (CMX_GEMM_STREAM): GEMM tests, GEMM census A/B, bench A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r05_y.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r05_y.log; grep -E "^FAILED|Error" gpurun_out/pytest_r05_y.log | head -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/gemm_census.py --ab GEMM_STREAM=0,1024,512 > gpurun_out/census_r05_y.txt 2>&1 || exit 1
grep -v "Warning\|capture_end\|amdgpu.ids" gpurun_out/census_r05_y.txt | head -14
timeout -k 10 300 python3 scripts/gemm_census.py --ab GEMM_STREAM_BPC=4,3,2 > gpurun_out/census_r05_y2.txt 2>&1 || exit 1
grep -v "Warning\|capture_end\|amdgpu.ids" gpurun_out/census_r05_y2.txt | head -14
REPS=3 bash scripts/ab_env.sh base CMX_GEMM_STREAM=0 || exit 1
