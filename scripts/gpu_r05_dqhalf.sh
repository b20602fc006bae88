#!/bin/bash
# 32-query dQ workgroups for under-filled short-sequence grids (CMX_SRA_DQ_HALF): tests, standalone, bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "sra" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r05_dqhalf.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r05_dqhalf.log; grep -E "^FAILED" gpurun_out/pytest_r05_dqhalf.log | head -5
[ $rc -eq 0 ] || exit $rc
for v in 0 1; do echo "== CMX_SRA_DQ_HALF=$v"; CMX_SRA_DQ_HALF=$v timeout -k 10 120 python3 scripts/bench_sra.py || exit 1; done
REPS=3 bash scripts/ab_env.sh base CMX_SRA_DQ_HALF=0 || exit 1
