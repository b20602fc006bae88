#!/bin/bash
# FRM channel-MLP backward with batched weight-row loads: module parity, bench, step census.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_x}
timeout -k 10 600 python -u -m pytest tests/test_gpu_modules.py tests/test_gpu_improved.py -m gpu -q --timeout 200 \
  --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
REPS=3 STEPS=30 bash scripts/ab_env.sh base > gpurun_out/ab_$TAG.txt 2>&1
rc=$?; cat gpurun_out/ab_$TAG.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 10 --warmup 2 \
  --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || exit $?
db=$(ls gpurun_out/prof_$TAG/*.db gpurun_out/prof_$TAG/*/*.db 2>/dev/null | head -1)
python3 scripts/step_census.py $db 200 > gpurun_out/step_census_$TAG.txt 2>&1
head -3 gpurun_out/step_census_$TAG.txt; grep "linear_" gpurun_out/step_census_$TAG.txt
rm -f $db
