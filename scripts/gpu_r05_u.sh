#!/bin/bash
# merged SRA backward launch (dQ + dK / dV in one grid): kernel tests, standalone A/B, bench A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "sra" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r05_u.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r05_u.log; grep -E "^FAILED|Error" gpurun_out/pytest_r05_u.log | head -5
[ $rc -eq 0 ] || exit $rc
for m in 1 0; do
  echo "== CMX_SRA_BWD_MERGED=$m"
  CMX_SRA_BWD_MERGED=$m timeout -k 10 120 python3 scripts/bench_sra.py || exit 1
done
REPS=3 bash scripts/ab_env.sh base CMX_SRA_BWD_MERGED=0 || exit 1
