#!/bin/bash
# write-through stores: kernel tests on the WT library, then interleaved bench A/B against the
# plain-store build (CMX_LIB_VARIANT=nowt)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_dwconv.py tests/test_gpu_kernels.py tests/test_gpu_optim.py \
  tests/test_gpu_grouped.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r04_e.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r04_e.log; [ $rc -eq 0 ] || exit $rc
REPS=3 bash scripts/ab_env.sh base "CMX_LIB_VARIANT=nowt" > gpurun_out/ab_r04_e.txt 2>&1; rc=$?
cat gpurun_out/ab_r04_e.txt; exit $rc
