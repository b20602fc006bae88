#!/bin/bash
# SQ counter passes on the SRA kernels (stages 1, 3, 4) and the step's GEMM / DW / LN kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_e}
SQ="SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_LDS"
for st in 1 3 4; do
  timeout -s KILL 120 rocprofv3 --pmc $SQ -d /tmp/sq_${TAG}_s$st -o run -- python3 scripts/bench_sra.py stage $st \
    > gpurun_out/sq_${TAG}_s$st.log 2>&1
  echo "sra stage $st rc=$?"
  python3 scripts/sq_summary.py $(ls /tmp/sq_${TAG}_s$st/*.db /tmp/sq_${TAG}_s$st/*/*.db 2>/dev/null | head -1) sra \
    > gpurun_out/sq_${TAG}_s$st.txt 2>&1
done
timeout -s KILL 200 rocprofv3 --pmc $SQ --kernel-include-regex "gemm_bf16|dw2|ln_" -d /tmp/sq_${TAG}_step -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sq_${TAG}_step.log 2>&1
echo "step rc=$?"
python3 scripts/sq_summary.py $(ls /tmp/sq_${TAG}_step/*.db /tmp/sq_${TAG}_step/*/*.db 2>/dev/null | head -1) \
  > gpurun_out/sq_${TAG}_step.txt 2>&1
ls -la gpurun_out/sq_${TAG}_*; head -30 gpurun_out/sq_${TAG}_s4.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_modules.py tests/test_gpu_gemm.py tests/test_config_parity.py -m gpu -v \
  --timeout 300 --timeout-method thread -k "ffm or h2 or config2 or config1" > gpurun_out/pytest_ffm_$TAG.log 2>&1
rc=$?; echo "pytest ffm rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/pytest_ffm_$TAG.log | tail -8
for arm in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_${arm}_$TAG.json 2>&1 || exit $?
  echo "bench $(grep -o '"value": [0-9.]*' gpurun_out/bench_${arm}_$TAG.json)"
done
timeout -k 10 400 python3 -u scripts/gemm_census.py --ab GEMM_DIRECT=0,1 > gpurun_out/ab_direct_$TAG.txt 2>&1 || exit $?
head -30 gpurun_out/ab_direct_$TAG.txt
