#!/bin/bash
# 64 x 128 tiles for wide short-K GEMMs (CMX_GEMM_WIDEN): GEMM parity under the knob, the
# per-shape probe, then the step A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_t}
CMX_GEMM_WIDEN=256 timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py -m gpu -q --timeout 200 \
  --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/gemm_probe.py GEMM_WIDEN=0,128,256,512 > gpurun_out/probe_$TAG.txt 2>&1
rc=$?; cat gpurun_out/probe_$TAG.txt; [ $rc -eq 0 ] || exit $rc
REPS=3 STEPS=30 bash scripts/ab_env.sh base "CMX_GEMM_WIDEN=512" "CMX_GEMM_WIDEN=256" > gpurun_out/ab_$TAG.txt 2>&1
rc=$?; cat gpurun_out/ab_$TAG.txt; [ $rc -eq 0 ] || exit $rc
