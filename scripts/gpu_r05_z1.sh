#!/bin/bash
# streaming GEMM grid on by default: GEMM tests, model / config parity, train tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_gemm.py tests/test_model_parity.py tests/test_config_parity.py tests/test_gpu_train.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/pytest_r05_z1.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r05_z1.log; grep -E "^FAILED|Error" gpurun_out/pytest_r05_z1.log | head -5
exit $rc
