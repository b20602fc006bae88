#!/bin/bash
# Kernel-traced bench per environment arm, keeping each arm's trace database for offline census /
# step traces (scripts/step_census.py, scripts/step_trace.py):
#   bash scripts/trace_ab.sh TAG base "CMX_FFM_STREAM=0"   ->  gpurun_out/tab_TAG_<i>/run_results.db
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
i=0
for arm in "$@"; do
  envs=""; [ "$arm" != "base" ] && envs="$arm"
  d=gpurun_out/tab_${TAG}_$i
  env $envs timeout -k 10 200 rocprofv3 --kernel-trace -d $d -o run -- python3 bench.py --steps 12 --warmup 3 \
    --no-cpu-baseline > $d.log 2>&1 || { echo "arm '$arm' failed"; tail -5 $d.log; exit 1; }
  db=$(ls $d/run_results.db $d/*/run_results.db 2>/dev/null | head -1)
  echo "[$i: $arm] $(python3 scripts/step_census.py $db 5 | sed -n 1,3p)"
  grep -o '"value": [0-9.]*' $d.log | head -1
  i=$((i + 1))
done
