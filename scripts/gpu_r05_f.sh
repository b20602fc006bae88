#!/bin/bash
# round-5 check: norm1 backward in the SR patch dgrad, FRM two-gradient combine, SRA forward threshold
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_modules.py tests/test_gpu_kernels.py -k "ln_tail or ln_bwd or frm or sra" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r05_f0.log 2>&1
rc=$?; echo "pytest kernels rc=$rc"; tail -3 gpurun_out/pytest_r05_f0.log; grep -E "^FAILED|Error" gpurun_out/pytest_r05_f0.log | head -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_model_parity.py tests/test_config_parity.py tests/test_gpu_train.py tests/test_gpu_fusion_local.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r05_f.log 2>&1
rc=$?; echo "pytest model rc=$rc"; tail -3 gpurun_out/pytest_r05_f.log; grep -E "^FAILED|Error" gpurun_out/pytest_r05_f.log | head -5
[ $rc -eq 0 ] || exit $rc
REPS=3 bash scripts/ab_env.sh base CMX_LN_BWD_FUSE=0
