#!/bin/bash
# One SQ counter pass (wave cycles split into waiting / issue-stalled / active, instruction mix)
# over a short bench run, kernels filtered by regex; per-kernel averages per dispatch.
#   bash scripts/pmc_sq.sh TAG REGEX
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}; RE=${2:?regex}
mkdir -p gpurun_out/profiles
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace --kernel-include-regex "$RE" -d gpurun_out/pmc_sq_$TAG -o run \
  -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_sq_$TAG.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/sq_table.py $(ls gpurun_out/pmc_sq_$TAG/*.db gpurun_out/pmc_sq_$TAG/*/*.db 2>/dev/null | head -1) \
  > gpurun_out/profiles/${TAG}_sq.txt 2>&1
cat gpurun_out/profiles/${TAG}_sq.txt
rm -rf gpurun_out/pmc_sq_$TAG
