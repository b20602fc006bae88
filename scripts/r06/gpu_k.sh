#!/bin/bash
# round-6: stage-3 SRA backward on the general kernels (CMX_SRA_SMALL_N below 1200) vs the short-sequence ones
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
for v in 2048 1000; do
  CMX_SRA_SMALL_N=$v timeout -k 10 120 python3 scripts/bench_sra.py > gpurun_out/r06/k_sra_$v.txt 2>&1
  rc=$?; echo "sra small_n=$v rc=$rc"; cat gpurun_out/r06/k_sra_$v.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
done
for v in 1000 2048 1000 2048; do
  CMX_SRA_SMALL_N=$v CMX_BENCH_NO_ROOFLINE=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r06/k_bench_$v.json 2> gpurun_out/r06/k_bench_$v.err
  rc=$?; echo "bench small_n=$v rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r06/k_bench_$v.json)"; [ $rc -eq 0 ] || exit $rc
done
