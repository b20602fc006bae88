#!/bin/bash
# round-6: one-launch small-map BatchNorm -- unit parity, standalone timings, model tests, bench A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_kernels.py -m gpu -k "batchnorm" > gpurun_out/r06/j_unit.log 2>&1
rc=$?; echo "unit rc=$rc"; tail -2 gpurun_out/r06/j_unit.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r06/j_unit.log | head -20; exit $rc; }
timeout -k 10 120 python3 scripts/bench_ops.py bnsmall > gpurun_out/r06/j_ops.txt 2>&1
rc=$?; echo "ops rc=$rc"; grep bn gpurun_out/r06/j_ops.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 $T tests/test_model_parity.py tests/test_gpu_train.py tests/test_gpu_modules.py -m gpu > gpurun_out/r06/j_model.log 2>&1
rc=$?; echo "model rc=$rc"; tail -2 gpurun_out/r06/j_model.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r06/j_model.log | head -20; exit $rc; }
for v in 600 0 600 0; do
  CMX_BN_SMALL_M=$v CMX_BENCH_NO_ROOFLINE=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r06/j_bench_$v.json 2> gpurun_out/r06/j_bench_$v.err
  rc=$?; echo "bench bnsmall=$v rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r06/j_bench_$v.json)"; [ $rc -eq 0 ] || exit $rc
done
