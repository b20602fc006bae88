#!/bin/bash
# the full GPU test suite as the driver runs it (one process), log under gpurun_out/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-suite}
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_$TAG.log; grep -E "^FAILED|^ERROR" gpurun_out/pytest_gpu_$TAG.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
