#!/bin/bash
# streaming GEMM grid at 5 resident blocks per CU (registers capped at 96, libcmx_hip_s5.so) vs 4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CMX_LIB_VARIANT=s5 timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -k "stream or ln_tail" -x -q --timeout 200 --timeout-method thread 2>&1 | tail -2
for r in 1 2; do
  timeout -k 10 300 python3 scripts/gemm_census.py --ab GEMM_STREAM=0,1024 2>/dev/null | grep "gemm calls" | sed "s/^/lb4 rep $r: /"
  CMX_LIB_VARIANT=s5 timeout -k 10 300 python3 scripts/gemm_census.py --ab GEMM_STREAM=0,1024 2>/dev/null | grep "gemm calls" | sed "s/^/lb5 rep $r: /"
done
REPS=3 bash scripts/ab_env.sh base CMX_LIB_VARIANT=s5 || exit 1
