#!/bin/bash
# round-5 check: new GPU tests (LN tail, segment update overlap) + interleaved A/B of the two switches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_optim.py tests/test_gpu_grouped.py tests/test_gpu_train.py tests/test_model_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r05_d.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r05_d.log; grep -E "^FAILED|Error" gpurun_out/pytest_r05_d.log | head -5
[ $rc -eq 0 ] || exit $rc
REPS=2 bash scripts/ab_env.sh base "CMX_OPT_OVERLAP=0" "CMX_LN_TAIL=0" "CMX_OPT_OVERLAP=0 CMX_LN_TAIL=0" "CMX_SIDE_WGRAD_BLOCKS=128 CMX_SIDE_ADAMW_BLOCKS=128"
