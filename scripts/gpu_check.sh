#!/bin/bash
# GPU-box routine: parity tests, bench line, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash/timeout (anything but pytest's exit 1 =
# "tests failed") ends the script so nothing else touches the GPU after a fault.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r01}
timeout -k 10 840 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
