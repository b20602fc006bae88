#!/bin/bash
# Round-4 probe of the fresh-box bench: the bench as the FIRST GPU process of the lease (as the
# driver runs it) with the per-replay device-time series and sysfs clocks, then a kernel trace
# of the same command, then the bench again.  Usage: bash scripts/gpu_fresh_probe.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r04_a}
CMX_BENCH_TRACE=300 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
  > gpurun_out/fresh_${TAG}_1.json 2> gpurun_out/fresh_${TAG}_1.err || exit $?
cut -c1-200 gpurun_out/fresh_${TAG}_1.json; grep -v amdgpu.ids gpurun_out/fresh_${TAG}_1.err | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 20 --warmup 5 \
  --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || exit $?
db=$(ls gpurun_out/prof_$TAG/*.db gpurun_out/prof_$TAG/*/*.db 2>/dev/null | head -1)
python3 scripts/step_series.py $db 3 > gpurun_out/step_series_$TAG.txt 2>&1
python3 scripts/step_census.py $db 60 > gpurun_out/step_census_$TAG.txt 2>&1
rm -f $db
CMX_BENCH_TRACE=300 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
  > gpurun_out/fresh_${TAG}_3.json 2> gpurun_out/fresh_${TAG}_3.err || exit $?
cut -c1-200 gpurun_out/fresh_${TAG}_3.json; grep -v amdgpu.ids gpurun_out/fresh_${TAG}_3.err | cut -c1-400
