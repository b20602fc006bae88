#!/bin/bash
# bilinear adjoint with 32-bit index arithmetic: fused-decoder / kernel parity, step census.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_bl}
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_kernels.py tests/test_gpu_train.py -m gpu -q \
  --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 10 --warmup 2 \
  --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || exit $?
db=$(ls gpurun_out/prof_$TAG/*.db gpurun_out/prof_$TAG/*/*.db 2>/dev/null | head -1)
python3 scripts/step_census.py $db 200 > gpurun_out/step_census_$TAG.txt 2>&1
head -1 gpurun_out/step_census_$TAG.txt; grep "bilinear" gpurun_out/step_census_$TAG.txt
rm -f $db
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2>/dev/null || exit $?
grep -o '"value": [0-9.]*' gpurun_out/bench_$TAG.json
