#!/bin/bash
# Register-streamed GEMM (CMX_GEMM_REG): tests, probe, step A/B (+ LN fusion widths).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_k}
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_train.py -m gpu -q --timeout 200 \
  --timeout-method thread -k "reg or ln_" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; grep -E "^FAILED" gpurun_out/pytest_$TAG.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/gemm_probe.py GEMM_REG=0,1 GEMM_REG_BPC=3,4 > gpurun_out/probe_$TAG.txt 2>&1 || exit $?
cat gpurun_out/probe_$TAG.txt
REPS=3 STEPS=30 bash scripts/ab_env.sh base "CMX_GEMM_REG=4096" "CMX_GEMM_REG=16384" \
  > gpurun_out/ab_$TAG.txt 2>&1
rc=$?; cat gpurun_out/ab_$TAG.txt; [ $rc -eq 0 ] || exit $rc
