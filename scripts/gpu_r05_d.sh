#!/bin/bash
# round-5 check: row-LayerNorm GEMM epilogue (kernel test, model / config parity), then A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -k "ln_tail or ln_bwd" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05_d0.log 2>&1
rc=$?; echo "pytest kernels rc=$rc"; tail -3 gpurun_out/pytest_r05_d0.log; grep -E "^FAILED|Error" gpurun_out/pytest_r05_d0.log | head -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_model_parity.py tests/test_config_parity.py tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r05_d.log 2>&1
rc=$?; echo "pytest model rc=$rc"; tail -3 gpurun_out/pytest_r05_d.log; grep -E "^FAILED|Error" gpurun_out/pytest_r05_d.log | head -5
[ $rc -eq 0 ] || exit $rc
REPS=3 bash scripts/ab_env.sh base CMX_LN_BWD_FUSE=0
