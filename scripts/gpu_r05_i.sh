#!/bin/bash
# two kept kernel traces of the default step (idle-gap variance between runs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
KEEP="0 1" bash scripts/trace_ab.sh r05_i base base || exit 1
for i in 0 1; do
  db=$(ls gpurun_out/tab_r05_i_$i/run_results.db gpurun_out/tab_r05_i_$i/*/run_results.db 2>/dev/null | head -1)
  python3 scripts/step_trace.py $db --gaps 8 > gpurun_out/r05_i_gaps_$i.txt
  python3 scripts/step_trace.py $db > gpurun_out/r05_i_trace_$i.txt
  cat gpurun_out/r05_i_gaps_$i.txt
done
REPS=3 bash scripts/ab_env.sh base CMX_FFM_STREAM=0
