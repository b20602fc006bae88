#!/bin/bash
# SQ counter passes on the short-sequence SRA kernels and the stage-1 GEMMs; direct-epilogue A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_e}
SQ="SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_LDS"
for st in 1 3 4; do
  timeout -s KILL 120 rocprofv3 --pmc $SQ -d gpurun_out/sq_${TAG}_s$st -o run -- python3 scripts/bench_sra.py stage $st \
    > gpurun_out/sq_${TAG}_s$st.log 2>&1 || exit $?
  python3 scripts/sq_summary.py $(ls gpurun_out/sq_${TAG}_s$st/*.db gpurun_out/sq_${TAG}_s$st/*/*.db 2>/dev/null | head -1) sra \
    > gpurun_out/sq_${TAG}_s$st.txt 2>&1
done
timeout -s KILL 200 rocprofv3 --pmc $SQ --kernel-include-regex "gemm_bf16|dw2|ln_" -d gpurun_out/sq_${TAG}_step -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sq_${TAG}_step.log 2>&1 || exit $?
python3 scripts/sq_summary.py $(ls gpurun_out/sq_${TAG}_step/*.db gpurun_out/sq_${TAG}_step/*/*.db 2>/dev/null | head -1) \
  > gpurun_out/sq_${TAG}_step.txt 2>&1
for arm in 0 1 0 1; do
  CMX_GEMM_DIRECT=$arm timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_direct${arm}_$TAG.json 2>&1 || exit $?
  echo "direct=$arm $(grep -o '"value": [0-9.]*' gpurun_out/ab_direct${arm}_$TAG.json)"
done
CMX_GEMM_DIRECT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py tests/test_model_parity.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "epilogue or layouts or two_segment or unaligned or eval_logits" \
  > gpurun_out/pytest_direct_$TAG.log 2>&1
echo "pytest direct rc=$?"; tail -2 gpurun_out/pytest_direct_$TAG.log
