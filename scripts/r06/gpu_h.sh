#!/bin/bash
# round-6: CE cells kernel -- unit parity, standalone timings, step bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_kernels.py -m gpu -k "upsample_ce" > gpurun_out/r06/h_ce.log 2>&1
rc=$?; echo "ce unit rc=$rc"; tail -3 gpurun_out/r06/h_ce.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r06/h_ce.log | head -20; exit $rc; }
timeout -k 10 120 python3 scripts/bench_ops.py ce > gpurun_out/r06/h_ce_ops.txt 2>&1
rc=$?; echo "ops rc=$rc"; cat gpurun_out/r06/h_ce_ops.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 $T tests/test_gpu_fused.py tests/test_gpu_train.py -m gpu > gpurun_out/r06/h_train.log 2>&1
rc=$?; echo "train rc=$rc"; tail -2 gpurun_out/r06/h_train.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r06/h_train.log | head; exit $rc; }
for i in 1 2; do
  CMX_BENCH_NO_ROOFLINE=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r06/h_bench$i.json 2> gpurun_out/r06/h_bench$i.err
  rc=$?; echo "bench rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r06/h_bench$i.json)"; [ $rc -eq 0 ] || exit $rc
done
