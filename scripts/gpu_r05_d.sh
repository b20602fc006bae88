#!/bin/bash
# round-5 check: new GPU tests (LN tail, Mix-FFN bands, segment update overlap) + interleaved A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mixffn.py tests/test_gpu_gemm.py -k "mixffn or ln_tail" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05_d0.log 2>&1
rc=$?; echo "pytest kernels rc=$rc"; tail -3 gpurun_out/pytest_r05_d0.log; grep -E "^FAILED|Error" gpurun_out/pytest_r05_d0.log | head -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_grouped.py tests/test_gpu_train.py tests/test_model_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r05_d.log 2>&1
rc=$?; echo "pytest model rc=$rc"; tail -3 gpurun_out/pytest_r05_d.log; grep -E "^FAILED|Error" gpurun_out/pytest_r05_d.log | head -5
[ $rc -eq 0 ] || exit $rc
REPS=2 bash scripts/ab_env.sh base "CMX_OPT_OVERLAP=0" "CMX_LN_TAIL=0" "CMX_MIXFFN=0" "CMX_OPT_OVERLAP=0 CMX_LN_TAIL=0 CMX_MIXFFN=0"
