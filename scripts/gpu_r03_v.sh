#!/bin/bash
# Host-side cost of a step: the host time to enqueue K graph replays against their GPU time.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_v}
for k in 10 40; do
  timeout -k 10 200 python -u bench.py --steps $k --warmup 5 --no-cpu-baseline > gpurun_out/bench_${TAG}_$k.json 2> gpurun_out/bench_${TAG}_$k.err || exit $?
  grep "host enqueue" gpurun_out/bench_${TAG}_$k.err; grep -o '"value": [0-9.]*' gpurun_out/bench_${TAG}_$k.json
done
