#!/bin/bash
# A/B routine of this round's kernel changes: parity tests of the touched kernels, standalone
# kernel timings, then bench lines per knob value (every GPU step under its own time limit).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
CMX_SRA_DKV_DIRECT=100000 $T tests/test_gpu_kernels.py tests/test_gpu_improved.py > gpurun_out/pt_a.log 2>&1; rc=$?; tail -2 gpurun_out/pt_a.log; [ $rc -le 1 ] || exit $rc
for v in 0 300 1200 4800; do echo "CMX_SRA_DKV_DIRECT=$v"; CMX_SRA_DKV_DIRECT=$v timeout -k 10 120 python -u scripts/bench_sra.py 2>/dev/null || exit 1; done
STEPS=60 VAR=CMX_SRA_DKV_DIRECT VALUES="0 300 1200 0 300 1200" bash scripts/env_sweep.sh
