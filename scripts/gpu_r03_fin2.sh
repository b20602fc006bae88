#!/bin/bash
# CE variant check, then the full GPU suite, the bench line and a step census of the tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_zy}
bash scripts/gpu_r03_ce2.sh ${TAG}_ce || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu_$TAG.log; grep -E "^FAILED" gpurun_out/pytest_gpu_$TAG.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 10 --warmup 2 \
  --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || exit $?
db=$(ls gpurun_out/prof_$TAG/*.db gpurun_out/prof_$TAG/*/*.db 2>/dev/null | head -1)
python3 scripts/step_census.py $db 200 > gpurun_out/step_census_$TAG.txt 2>&1
head -3 gpurun_out/step_census_$TAG.txt; grep "ce_\|linear_bwd" gpurun_out/step_census_$TAG.txt
rm -f $db
