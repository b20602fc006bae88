#!/bin/bash
# round-6: one-launch BN threshold 2400 (stage 3 too) vs 600, 3 interleaved pairs after a throwaway run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > /dev/null 2>&1 || exit 1
for v in 2400 600 2400 600 2400 600; do
  CMX_BN_SMALL_M=$v CMX_BENCH_NO_ROOFLINE=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r06/l_bench_$v.json 2> gpurun_out/r06/l_bench_$v.err
  rc=$?; echo "bench bnsmall=$v rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r06/l_bench_$v.json)"; [ $rc -eq 0 ] || exit $rc
done
