#!/bin/bash
# HIP hardware-queue count per process vs the step (interleaved, twice)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 100 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > /dev/null 2>&1
for r in 1 2; do
  for q in 4 1 2 3; do
    GPU_MAX_HW_QUEUES=$q CMX_BENCH_NO_ROOFLINE=1 timeout -k 10 150 python3 bench.py --steps 12 --warmup 3 --no-cpu-baseline > gpurun_out/hwq_$q.json 2> gpurun_out/hwq_$q.err
    echo "hwq$q $r rc=$? $(grep -o '"value": [0-9.]*' gpurun_out/hwq_$q.json)"
    [ -s gpurun_out/hwq_$q.json ] || tail -3 gpurun_out/hwq_$q.err
  done
done
