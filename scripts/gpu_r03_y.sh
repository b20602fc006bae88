#!/bin/bash
# BatchNorm row-block cap (CMX_BN_NBLK): BN parity at the cap, per-arm BN kernel census, step A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_y}
CMX_BN_NBLK=1024 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q --timeout 200 \
  --timeout-method thread -k "batchnorm" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
for nb in 256 512 1024; do
  CMX_BN_NBLK=$nb timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_${TAG}_$nb -o run -- python3 bench.py \
    --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_${TAG}_$nb.log 2>&1 || exit $?
  db=$(ls gpurun_out/prof_${TAG}_$nb/*.db gpurun_out/prof_${TAG}_$nb/*/*.db 2>/dev/null | head -1)
  python3 scripts/step_census.py $db 200 > gpurun_out/step_census_${TAG}_$nb.txt 2>&1
  echo "BN_NBLK=$nb"; head -1 gpurun_out/step_census_${TAG}_$nb.txt; grep " bn_" gpurun_out/step_census_${TAG}_$nb.txt
  rm -f $db
done
REPS=3 STEPS=30 bash scripts/ab_env.sh base "CMX_BN_NBLK=512" "CMX_BN_NBLK=1024" > gpurun_out/ab_$TAG.txt 2>&1
rc=$?; cat gpurun_out/ab_$TAG.txt; [ $rc -eq 0 ] || exit $rc
