#!/bin/bash
# round-6: CE tile loads in flight together -- CE tests, step A/B against the previous commit (old)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  tests/test_gpu_fused.py tests/test_model_parity.py > gpurun_out/r06/ce_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r06/ce_tests.log; grep -E "^FAILED" gpurun_out/r06/ce_tests.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 scripts/bench_ops.py ce > gpurun_out/r06/ce_ops_new.txt 2>&1 && CMX_LIB_VARIANT=old timeout -k 10 120 python3 scripts/bench_ops.py ce > gpurun_out/r06/ce_ops_old.txt 2>&1 || exit 1
grep -h "us" gpurun_out/r06/ce_ops_new.txt gpurun_out/r06/ce_ops_old.txt
REPS=${REPS:-3} bash scripts/ab_env.sh base "CMX_LIB_VARIANT=old"
