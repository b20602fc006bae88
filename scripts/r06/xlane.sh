#!/bin/bash
# round-6: DPP / permlane cross-lane reductions -- lane-exchange probe, the GPU suite, step A/B
# against the previous library (CMX_LIB_VARIANT=old)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/xor_lane_probe.hip -o /tmp/xor_lane_probe 2>/dev/null || { echo "probe build failed"; exit 1; }
timeout -k 10 60 /tmp/xor_lane_probe || exit 1
[ "${SUITE:-1}" = 1 ] && { bash scripts/gpu_suite.sh xlane || exit 1; }
REPS=${REPS:-3} bash scripts/ab_env.sh base "CMX_LIB_VARIANT=old"
