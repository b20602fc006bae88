#!/bin/bash
# Longest-first grouped weight-gradient records (CMX_GROUPED_SORT), FFM side stream on/off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_n}
CMX_GROUPED_SORT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_optim.py -m gpu -q \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; grep -E "^FAILED" gpurun_out/pytest_$TAG.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
REPS=3 STEPS=30 bash scripts/ab_env.sh base "CMX_GROUPED_SORT=1" "CMX_FFM_STREAM=0" > gpurun_out/ab_$TAG.txt 2>&1
rc=$?; cat gpurun_out/ab_$TAG.txt; [ $rc -eq 0 ] || exit $rc
