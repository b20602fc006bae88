#!/bin/bash
# graph executor streams = 2: interleaved A/B (3 pairs) and a kept trace of each arm
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
REPS=3 bash scripts/ab_env.sh base DEBUG_HIP_FORCE_GRAPH_QUEUES=2 || exit 1
KEEP="0 1" bash scripts/trace_ab.sh r05_p base DEBUG_HIP_FORCE_GRAPH_QUEUES=2 || exit 1
for i in 0 1; do
  db=$(ls gpurun_out/tab_r05_p_$i/run_results.db gpurun_out/tab_r05_p_$i/*/run_results.db 2>/dev/null | head -1)
  python3 scripts/step_trace.py $db > gpurun_out/r05_p_trace_$i.txt
  python3 scripts/step_trace.py $db --gaps 5 | head -30
  rm -rf gpurun_out/tab_r05_p_$i
done
