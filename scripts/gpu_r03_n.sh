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
SQ="SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_LDS"
timeout -s KILL 120 rocprofv3 --pmc $SQ -d gpurun_out/sq_$TAG -o run -- python3 scripts/bench_sra.py stage 1 \
  > gpurun_out/sq_$TAG.log 2>&1
echo "sq rc=$?"
python3 scripts/sq_summary.py $(ls gpurun_out/sq_$TAG/*.db gpurun_out/sq_$TAG/*/*.db 2>/dev/null | head -1) sra \
  > gpurun_out/sq_sra_$TAG.txt 2>&1
cat gpurun_out/sq_sra_$TAG.txt | head -20
rm -rf gpurun_out/sq_$TAG
