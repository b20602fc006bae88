#!/bin/bash
# SQ counters of the fused upsample + CE backward (standalone, scripts/bench_ops.py ce).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_ce}
timeout -k 10 120 python3 scripts/bench_ops.py ce > gpurun_out/ce_$TAG.txt 2>&1 || exit $?
cat gpurun_out/ce_$TAG.txt
P1="SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT,SQ_INSTS_SALU,SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_VALU,SQ_INSTS_SMEM"
n=0
for P in $P1 $P2; do
  n=$((n + 1))
  timeout -s KILL 60 rocprofv3 --pmc $P -d gpurun_out/sq_${TAG}_$n -o run -- python3 scripts/bench_ops.py ce \
    > gpurun_out/sq_${TAG}_$n.log 2>&1 || { echo "pass $n failed"; tail -3 gpurun_out/sq_${TAG}_$n.log; exit 1; }
  python3 scripts/sq_summary.py $(ls gpurun_out/sq_${TAG}_$n/*.db gpurun_out/sq_${TAG}_$n/*/*.db 2>/dev/null | head -1) ce_ \
    > gpurun_out/sq_ce_${TAG}_$n.txt 2>&1
  cat gpurun_out/sq_ce_${TAG}_$n.txt
  rm -rf gpurun_out/sq_${TAG}_$n
done
