#!/bin/bash
# A/B routine of this round's kernel changes: parity tests of the touched kernels, standalone
# kernel timings, then bench lines per knob value (every GPU step under its own time limit).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
$T tests/test_gpu_gemm.py tests/test_gpu_dwconv.py tests/test_gpu_grouped.py tests/test_gpu_kernels.py > gpurun_out/pt_a.log 2>&1; rc=$?; tail -2 gpurun_out/pt_a.log; [ $rc -le 1 ] || exit $rc
CMX_GEMM_KW=4 $T tests/test_gpu_gemm.py > gpurun_out/pt_b.log 2>&1; rc=$?; tail -2 gpurun_out/pt_b.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u scripts/bench_dw.py || exit 1
timeout -k 10 120 python -u scripts/bench_sra.py || exit 1
CMX_GEMM_KW=4 timeout -k 10 200 python -u scripts/gemm_sweep.py || exit 1
STEPS=60 VAR=CMX_GEMM_KW VALUES="2 4 2 4" bash scripts/env_sweep.sh
