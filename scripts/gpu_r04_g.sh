#!/bin/bash
# module + train tests of this round's changes, then the graph-launch env A/B (host enqueue)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_modules.py tests/test_gpu_train.py tests/test_gpu_optim.py tests/test_gpu_improved.py \
  -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r04_g.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r04_g.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r04_f.sh
