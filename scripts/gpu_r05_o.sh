#!/bin/bash
# HIP graph executor streams (DEBUG_HIP_FORCE_GRAPH_QUEUES) vs the step, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
REPS=2 STEPS=20 bash scripts/ab_env.sh base DEBUG_HIP_FORCE_GRAPH_QUEUES=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=2 DEBUG_HIP_FORCE_GRAPH_QUEUES=3 GPU_STREAMOPS_CP_WAIT=1
