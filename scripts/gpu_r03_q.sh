#!/bin/bash
# BN backward reduce at two rows per lane (151 VGPRs, 3 waves / SIMD instead of 256 / 1): BN tests, bench x3, census.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_q}
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_modules.py -m gpu -q --timeout 200 \
  --timeout-method thread -k "bn or batchnorm or ffm or decoder" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; grep -E "^FAILED" gpurun_out/pytest_$TAG.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
REPS=3 STEPS=30 bash scripts/ab_env.sh base > gpurun_out/ab_$TAG.txt 2>&1
rc=$?; cat gpurun_out/ab_$TAG.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 5 --warmup 3 \
  --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || exit $?
db=$(ls gpurun_out/prof_$TAG/*.db gpurun_out/prof_$TAG/*/*.db 2>/dev/null | head -1)
python3 scripts/step_census.py $db 200 > gpurun_out/step_census_$TAG.txt 2>&1
grep -E "launches|bn_" gpurun_out/step_census_$TAG.txt | head
rm -rf gpurun_out/prof_$TAG
