#!/bin/bash
# write-through probe; AdamW (step ticket) tests; bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/wt_probe.py > gpurun_out/wt_probe.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/wt_probe.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_train.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r04_d.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r04_d.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_r04_d.json 2> gpurun_out/bench_r04_d.err || exit $?
cut -c1-200 gpurun_out/bench_r04_d.json
