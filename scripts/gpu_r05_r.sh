#!/bin/bash
# HIP graph runtime knobs on top of bench.py's 2 graph streams (interleaved, 2 reps)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
REPS=2 bash scripts/ab_env.sh base DEBUG_HIP_GRAPH_BATCH_SIZE=16 DEBUG_HIP_GRAPH_BATCH_SIZE=256 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 DEBUG_HIP_DYNAMIC_QUEUES=1
