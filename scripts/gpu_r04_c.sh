#!/bin/bash
# Round-4 diagnostics: one step's launch-by-launch trace, and SQ wave-cycle counters of the
# step's 64 x 64 GEMM tiles (where does a 7 us small GEMM spend its time).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r04_c}
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 10 --warmup 3 \
  --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || exit $?
db=$(ls gpurun_out/prof_$TAG/*.db gpurun_out/prof_$TAG/*/*.db 2>/dev/null | head -1)
python3 scripts/step_trace.py $db > gpurun_out/step_trace_$TAG.txt 2>&1
python3 scripts/step_census.py $db 200 > gpurun_out/step_census_$TAG.txt 2>&1
rm -rf gpurun_out/prof_$TAG
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES \
  SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "gemm_bf16_kernel|dw2_|ln_fwd|ln_bwd" -d gpurun_out/sq_$TAG -o run \
  -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sq_$TAG.log 2>&1 || exit $?
db=$(ls gpurun_out/sq_$TAG/*.db gpurun_out/sq_$TAG/*/*.db 2>/dev/null | head -1)
python3 scripts/sq_summary.py $db > gpurun_out/sq_summary_$TAG.txt 2>&1
rm -rf gpurun_out/sq_$TAG
head -50 gpurun_out/sq_summary_$TAG.txt
CMX_PARITY_DUMP=1 timeout -k 10 600 python -u -m pytest tests/test_config_parity.py -m gpu -x -q --timeout 580 \
  --timeout-method thread -k "config2_b2_480x640_bs2" > gpurun_out/parity_dump_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/parity_dump_$TAG.log; [ $rc -le 1 ] || exit $rc
ls -la gpurun_out/parity/
