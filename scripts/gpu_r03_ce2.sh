#!/bin/bash
# CE backward VALU trim: parity + standalone timing + VALU count.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_ce2}
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train.py -m gpu -q --timeout 200 \
  --timeout-method thread -k "upsample_ce or ce_ or loss" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 scripts/bench_ops.py ce > gpurun_out/ce_$TAG.txt 2>&1 || exit $?
cat gpurun_out/ce_$TAG.txt
P1="SQ_WAVES,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_LDS_BANK_CONFLICT"
timeout -s KILL 60 rocprofv3 --pmc $P1 -d gpurun_out/sq_${TAG} -o run -- python3 scripts/bench_ops.py ce \
  > gpurun_out/sq_${TAG}.log 2>&1 || { echo "pmc failed"; tail -3 gpurun_out/sq_${TAG}.log; exit 1; }
python3 scripts/sq_summary.py $(ls gpurun_out/sq_${TAG}/*.db gpurun_out/sq_${TAG}/*/*.db 2>/dev/null | head -1) ce_ \
  > gpurun_out/sq_ce_${TAG}.txt 2>&1
cat gpurun_out/sq_ce_${TAG}.txt
rm -rf gpurun_out/sq_${TAG}
