#!/bin/bash
# FRM multi-launch default restored; A/B of side-stream weight gradients and grouped ring depth;
# GEMM tile / epilogue probe; kernel census.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_i}
timeout -k 10 600 python -u -m pytest tests/test_gpu_modules.py tests/test_gpu_train.py tests/test_model_parity.py -m gpu \
  -v --timeout 300 --timeout-method thread -k "frm or side or segment or b0" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed|Error" gpurun_out/pytest_$TAG.log | tail -15
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
REPS=2 STEPS=20 bash scripts/ab_env.sh base "CMX_WGRAD_SIDE=1" "CMX_GROUPED_NS=3" "CMX_GROUPED_NS=4" \
  > gpurun_out/ab_$TAG.txt 2>&1; rc=$?; cat gpurun_out/ab_$TAG.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/gemm_probe.py GEMM_SMALLK=0,256 GEMM_DIRECT=0,1 > gpurun_out/probe_$TAG.txt 2>&1 || exit $?
cat gpurun_out/probe_$TAG.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 5 --warmup 3 \
  --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || exit $?
db=$(ls gpurun_out/prof_$TAG/*.db gpurun_out/prof_$TAG/*/*.db 2>/dev/null | head -1)
python3 scripts/step_census.py $db 200 > gpurun_out/step_census_$TAG.txt 2>&1
head -70 gpurun_out/step_census_$TAG.txt
rm -f $db
