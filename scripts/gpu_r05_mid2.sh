#!/bin/bash
# GEMM_MID default 50: GEMM / model / config parity tests, then bench pairs against 0
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_gemm.py tests/test_model_parity.py tests/test_config_parity.py tests/test_gpu_train.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/pytest_r05_mid2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r05_mid2.log; grep -E "^FAILED" gpurun_out/pytest_r05_mid2.log | head -5
[ $rc -eq 0 ] || exit $rc
REPS=3 bash scripts/ab_env.sh base CMX_GEMM_MID=0 || exit 1
