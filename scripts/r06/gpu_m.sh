#!/bin/bash
# round-6: AdamW step scalars once per workgroup -- optimizer tests, bench A/B (CMX_ADAMW_BS)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_optim.py tests/test_gpu_train.py -m gpu > gpurun_out/r06/m_optim.log 2>&1
rc=$?; echo "optim rc=$rc"; tail -2 gpurun_out/r06/m_optim.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r06/m_optim.log | head; exit $rc; }
for v in 1 0 1 0; do
  CMX_ADAMW_BS=$v CMX_BENCH_NO_ROOFLINE=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r06/m_bench_$v.json 2> gpurun_out/r06/m_bench_$v.err
  rc=$?; echo "bench adamw_bs=$v rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r06/m_bench_$v.json)"; [ $rc -eq 0 ] || exit $rc
done
