#!/bin/bash
# round-6: decoder upsample-sum / 3-grid adjoint -- unit parity, model tests, bench A/B (CMX_DECODER_ADJ3)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_fused.py -m gpu -k "decoder or up3" > gpurun_out/r06/i_unit.log 2>&1
rc=$?; echo "unit rc=$rc"; tail -3 gpurun_out/r06/i_unit.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r06/i_unit.log | head -20; exit $rc; }
timeout -k 10 600 $T tests/test_model_parity.py tests/test_gpu_train.py -m gpu > gpurun_out/r06/i_model.log 2>&1
rc=$?; echo "model rc=$rc"; tail -2 gpurun_out/r06/i_model.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r06/i_model.log | head -20; exit $rc; }
for v in 1 0 1 0; do
  CMX_DECODER_ADJ3=$v CMX_BENCH_NO_ROOFLINE=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r06/i_bench_adj3$v.json 2> gpurun_out/r06/i_bench_adj3$v.err
  rc=$?; echo "bench adj3=$v rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r06/i_bench_adj3$v.json)"; [ $rc -eq 0 ] || exit $rc
done
