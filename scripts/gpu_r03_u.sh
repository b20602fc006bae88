#!/bin/bash
# sra_dq_small at three waves per SIMD (CMX_SRA_DQ_MINB=3): SRA parity, standalone per-stage
# timing of both builds, step A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_u}
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q --timeout 200 \
  --timeout-method thread -k "sra" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
for mb in 1 3; do
  echo "SRA_DQ_MINB=$mb"; CMX_SRA_DQ_MINB=$mb timeout -k 10 200 python -u scripts/bench_sra.py 2>&1 | grep -v amdgpu.ids
done > gpurun_out/sra_$TAG.txt
rc=$?; cat gpurun_out/sra_$TAG.txt; [ $rc -eq 0 ] || exit $rc
REPS=3 STEPS=30 bash scripts/ab_env.sh base "CMX_SRA_DQ_MINB=3" > gpurun_out/ab_$TAG.txt 2>&1
rc=$?; cat gpurun_out/ab_$TAG.txt; [ $rc -eq 0 ] || exit $rc
