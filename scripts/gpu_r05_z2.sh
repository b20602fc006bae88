#!/bin/bash
# streaming GEMM grid on (default) vs off: 5 interleaved bench pairs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
REPS=5 bash scripts/ab_env.sh base CMX_GEMM_STREAM=0 || exit 1
