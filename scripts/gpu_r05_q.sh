#!/bin/bash
# bench.py's own graph-stream setting (2 for one GPU) against the runtime default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
REPS=3 bash scripts/ab_env.sh base CMX_GRAPH_STREAMS=0
