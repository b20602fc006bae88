#!/bin/bash
# LN-fused residual GEMM epilogue (cmx_gemm_ln) + deep LDS-DMA rings (CMX_GEMM_DEEP): tests, probe, step A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_j}
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_train.py -m gpu -q --timeout 200 \
  --timeout-method thread -k "ln_ or stream or step_shapes or epilogues" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; grep -E "^FAILED|Error" gpurun_out/pytest_$TAG.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
CMX_GEMM_DEEP=6 timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py -m gpu -q --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_deep_$TAG.log 2>&1
rc=$?; echo "pytest deep rc=$rc"; tail -2 gpurun_out/pytest_deep_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/gemm_probe.py GEMM_DEEP=0,3,4,6 > gpurun_out/probe_$TAG.txt 2>&1 || exit $?
cat gpurun_out/probe_$TAG.txt
REPS=2 STEPS=20 bash scripts/ab_env.sh base "CMX_LN_FUSE=0" "CMX_GEMM_DEEP=4" "CMX_GEMM_DEEP=6" > gpurun_out/ab_$TAG.txt 2>&1
rc=$?; cat gpurun_out/ab_$TAG.txt; [ $rc -eq 0 ] || exit $rc
