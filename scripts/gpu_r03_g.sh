#!/bin/bash
# Round-3 re-entry record: full GPU suite + bench + kernel trace (gpu_check.sh), then the
# config-5 fp16 + loss-scaling bench line and the input-pipeline throughput.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03_g}
bash scripts/gpu_check.sh $TAG || exit $?
timeout -k 10 300 python -u bench.py --backbone mit_b5 --height 1024 --width 1024 --batch 1 --classes 19 \
  --dtype float16 --loss-scaling --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c5_fp16_$TAG.json \
  2> gpurun_out/bench_c5_fp16_$TAG.err || exit $?
cat gpurun_out/bench_c5_fp16_$TAG.json
timeout -k 10 300 python -u scripts/bench_loader.py > gpurun_out/loader_$TAG.json 2> gpurun_out/loader_$TAG.err || exit $?
cat gpurun_out/loader_$TAG.json
