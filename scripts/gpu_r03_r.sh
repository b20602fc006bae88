#!/bin/bash
# LayerNorm backward launch shape A/B (CMX_LN_BWD_NB, CMX_LN_BWD_RPT).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_r}
CMX_LN_BWD_NB=384 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q --timeout 200 \
  --timeout-method thread -k "layernorm or ln" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
REPS=3 STEPS=30 bash scripts/ab_env.sh base "CMX_LN_BWD_NB=384" "CMX_LN_BWD_RPT=1" "CMX_LN_BWD_NB=256" > gpurun_out/ab_$TAG.txt 2>&1
rc=$?; cat gpurun_out/ab_$TAG.txt; [ $rc -eq 0 ] || exit $rc
