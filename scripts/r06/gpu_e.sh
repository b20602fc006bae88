#!/bin/bash
# round-6: decoder fold (DecoderFoldF) -- unit parity, model parity, bench A/B against CMX_DECODER_FOLD=0
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_fused.py -m gpu -k "decoder" > gpurun_out/r06/e_fold.log 2>&1
rc=$?; echo "fold unit rc=$rc"; tail -3 gpurun_out/r06/e_fold.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r06/e_fold.log | head -20; exit $rc; }
timeout -k 10 600 $T tests/test_model_parity.py tests/test_gpu_train.py tests/test_gpu_improved.py -m gpu > gpurun_out/r06/e_model.log 2>&1
rc=$?; echo "model rc=$rc"; tail -3 gpurun_out/r06/e_model.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r06/e_model.log | head -20; exit $rc; }
timeout -k 10 600 $T tests/test_config_parity.py -m gpu -k "config4" -s > gpurun_out/r06/e_par4.log 2>&1
rc=$?; echo "par4 rc=$rc"; grep -E "worst|PASS|FAIL" gpurun_out/r06/e_par4.log | head -5
for v in 1 0 1 0; do
  CMX_DECODER_FOLD=$v CMX_BENCH_NO_ROOFLINE=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r06/e_bench_fold$v.json 2> gpurun_out/r06/e_bench_fold$v.err
  rc=$?; echo "bench fold=$v rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r06/e_bench_fold$v.json)"; [ $rc -eq 0 ] || exit $rc
done
