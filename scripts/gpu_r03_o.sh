#!/bin/bash
# SRA launch shapes: short-sequence kernels at every stage (CMX_SRA_SMALL_N), two query
# sub-tiles per wave (CMX_SRA_QW) / 4-wave workgroups (CMX_SRA_NW): standalone + step A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_o}
for arm in "base" "CMX_SRA_SMALL_N=5000" "CMX_SRA_SMALL_N=20000" "CMX_SRA_QW=2" "CMX_SRA_QW=2 CMX_SRA_NW=4" "CMX_SRA_NW=4"; do
  echo "[$arm]" >> gpurun_out/sra_$TAG.txt
  envs=""; [ "$arm" != "base" ] && envs="$arm"
  env $envs timeout -k 10 200 python -u scripts/bench_sra.py >> gpurun_out/sra_$TAG.txt 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/sra_$TAG.txt
CMX_SRA_SMALL_N=20000 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q --timeout 200 \
  --timeout-method thread -k "sra" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest small rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
CMX_SRA_QW=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q --timeout 200 \
  --timeout-method thread -k "sra" > gpurun_out/pytest_qw_$TAG.log 2>&1
rc=$?; echo "pytest qw2 rc=$rc"; tail -2 gpurun_out/pytest_qw_$TAG.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
REPS=3 STEPS=30 bash scripts/ab_env.sh base "CMX_SRA_SMALL_N=20000" "CMX_SRA_QW=2" > gpurun_out/ab_$TAG.txt 2>&1
rc=$?; cat gpurun_out/ab_$TAG.txt; [ $rc -eq 0 ] || exit $rc
