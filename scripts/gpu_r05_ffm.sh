#!/bin/bash
# FFM branch on its own captured stream (default) vs on the main stream
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
REPS=3 bash scripts/ab_env.sh base CMX_FFM_STREAM=0 "CMX_FFM_STREAM=0 CMX_GRAPH_STREAMS=1" || exit 1
