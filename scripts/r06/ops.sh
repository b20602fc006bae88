#!/bin/bash
# round-6: standalone op timings (scripts/bench_ops.py NAME...)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 180 python3 scripts/bench_ops.py "$@" > gpurun_out/r06/ops.txt 2>&1
rc=$?; echo "ops rc=$rc"; cat gpurun_out/r06/ops.txt; exit $rc
