#!/bin/bash
# one-launch FRM channel kernels: module parity + graph replay, step bench, kernel trace census.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_f}
timeout -k 10 600 python -u -m pytest tests/test_gpu_modules.py tests/test_gpu_kernels.py tests/test_model_parity.py -m gpu -v --timeout 900 \
  --timeout-method thread -k "frm or sra or layernorm or (train_step and b0)" > gpurun_out/pytest_frm_$TAG.log 2>&1
rc=$?; echo "pytest frm rc=$rc"; grep -E "FAILED|passed|failed|Error" gpurun_out/pytest_frm_$TAG.log | tail -12
[ $rc -eq 0 ] || exit $rc
for st in 1 2 3 4; do
  timeout -k 10 120 python -u scripts/bench_sra.py stage $st >> gpurun_out/sra_$TAG.log 2>&1 || exit $?
done
grep "N=" gpurun_out/sra_$TAG.log
for arm in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_${arm}_$TAG.json 2>&1 || exit $?
  echo "bench $(grep -o '"value": [0-9.]*' gpurun_out/bench_${arm}_$TAG.json)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG -o run -- python3 bench.py --steps 5 --warmup 3 \
  --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || exit $?
db=$(ls /tmp/prof_$TAG/*.db /tmp/prof_$TAG/*/*.db 2>/dev/null | head -1)
python3 scripts/step_census.py $db 200 > gpurun_out/step_census_$TAG.txt 2>&1
head -50 gpurun_out/step_census_$TAG.txt
stats=$(ls /tmp/prof_$TAG/*kernel_stats.csv /tmp/prof_$TAG/*/*kernel_stats.csv 2>/dev/null | head -1)
[ -n "$stats" ] && cp "$stats" gpurun_out/kernel_stats_$TAG.csv
true
