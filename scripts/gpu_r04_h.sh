#!/bin/bash
# stage-1 direct patch-embed conv: kernel tests, train / parity tests, bench + kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r04_h
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_modules.py -k "pe1 or implicit or frm or ifrm or multi" -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_r04_h1.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r04_h1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py tests/test_config_parity.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_r04_h2.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r04_h2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/bench_sra.py nw > gpurun_out/sra_nw_r04_h.txt 2>&1
rc=$?; tail -3 gpurun_out/sra_nw_r04_h.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u bench.py --steps 40 --warmup 10 > gpurun_out/bench_r04_h.json 2> gpurun_out/bench_r04_h.err
rc=$?; tail -c 600 gpurun_out/bench_r04_h.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r04_h" -o run \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/prof_r04_h/bench.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
