#!/bin/bash
# round-5 check: fusion switch test, FRM/BN local parity tests, then a kept kernel trace of the
# default step (scripts/step_trace.py reads gpurun_out/tab_r05_g_0/*/run_results.db)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_fusion_local.py -k "fusion" -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_r05_g.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r05_g.log; grep -E "^FAILED|Error|passed|failed" gpurun_out/pytest_r05_g.log | head -12
[ $rc -eq 0 ] || exit $rc
KEEP="0" bash scripts/trace_ab.sh r05_g base
