#!/bin/bash
# round-5 check: Mix-FFN 2-D tiles at stages 1-2 (kernel tests, model / config parity), then A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_mixffn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05_l0.log 2>&1
rc=$?; echo "pytest kernels rc=$rc"; tail -3 gpurun_out/pytest_r05_l0.log; grep -E "^FAILED|Error" gpurun_out/pytest_r05_l0.log | head -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_model_parity.py tests/test_config_parity.py tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r05_l.log 2>&1
rc=$?; echo "pytest model rc=$rc"; tail -3 gpurun_out/pytest_r05_l.log; grep -E "^FAILED|Error" gpurun_out/pytest_r05_l.log | head -5
[ $rc -eq 0 ] || exit $rc
REPS=3 bash scripts/ab_env.sh base CMX_MIXFFN_TILE=0 || exit 1
REPS=1 bash scripts/ab_prof.sh "mixffn|dw2_|gemm_bf16_kernel<64, 64, false, false, 2, 1|gemm_bf16_kernel<64, 64, false, true, 2, 1" base CMX_MIXFFN_TILE=0
