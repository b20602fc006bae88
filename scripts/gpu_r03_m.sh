#!/bin/bash
# Two-batch stage-1 im2col (no image concat), key/value path on a side stream (CMX_SR_STREAM):
# model parity tests, step A/B, kernel census.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_m}
timeout -k 10 600 python -u -m pytest tests/test_model_parity.py tests/test_gpu_train.py tests/test_golden.py -m gpu -q \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; grep -E "^FAILED" gpurun_out/pytest_$TAG.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
CMX_SR_STREAM=1 timeout -k 10 600 python -u -m pytest tests/test_model_parity.py tests/test_gpu_train.py -m gpu -q \
  --timeout 300 --timeout-method thread -k "b0 or segment or side" > gpurun_out/pytest_sr_$TAG.log 2>&1
rc=$?; echo "pytest sr-stream rc=$rc"; tail -2 gpurun_out/pytest_sr_$TAG.log; grep -E "^FAILED" gpurun_out/pytest_sr_$TAG.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
REPS=3 STEPS=30 bash scripts/ab_env.sh base "CMX_SR_STREAM=1" > gpurun_out/ab_$TAG.txt 2>&1
rc=$?; cat gpurun_out/ab_$TAG.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 5 --warmup 3 \
  --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || exit $?
db=$(ls gpurun_out/prof_$TAG/*.db gpurun_out/prof_$TAG/*/*.db 2>/dev/null | head -1)
python3 scripts/step_census.py $db 200 > gpurun_out/step_census_$TAG.txt 2>&1
head -12 gpurun_out/step_census_$TAG.txt
rm -rf gpurun_out/prof_$TAG
