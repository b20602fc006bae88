#!/bin/bash
# is the kernel-traced bench faster than the plain one (same arguments)?  interleaved, twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 100 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > /dev/null 2>&1
for r in 1 2; do
  CMX_BENCH_NO_ROOFLINE=1 timeout -k 10 150 python3 bench.py --steps 12 --warmup 3 --no-cpu-baseline 2>/dev/null | grep -o '"value": [0-9.]*' | sed "s/^/plain $r /"
  CMX_BENCH_NO_ROOFLINE=1 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tj_$r -o run -- python3 bench.py --steps 12 --warmup 3 --no-cpu-baseline 2>/dev/null | grep -o '"value": [0-9.]*' | sed "s/^/traced $r /"
  rm -rf gpurun_out/tj_$r
  GPU_MAX_HW_QUEUES=2 CMX_BENCH_NO_ROOFLINE=1 timeout -k 10 150 python3 bench.py --steps 12 --warmup 3 --no-cpu-baseline 2>/dev/null | grep -o '"value": [0-9.]*' | sed "s/^/hwq2 $r /"
  GPU_MAX_HW_QUEUES=8 CMX_BENCH_NO_ROOFLINE=1 timeout -k 10 150 python3 bench.py --steps 12 --warmup 3 --no-cpu-baseline 2>/dev/null | grep -o '"value": [0-9.]*' | sed "s/^/hwq8 $r /"
done
