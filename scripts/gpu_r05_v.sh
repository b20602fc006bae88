#!/bin/bash
# BatchNorm in-kernel ticket fold: BN kernel tests, module / train tests, op timings, bench A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "batchnorm" tests/test_gpu_modules.py tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r05_v.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r05_v.log; grep -E "^FAILED|Error" gpurun_out/pytest_r05_v.log | head -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 scripts/bench_ops.py bn || exit 1
REPS=3 bash scripts/ab_env.sh base CMX_BN_TICKET_FOLD=0 || exit 1
