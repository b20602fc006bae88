#!/bin/bash
# runtime environment knobs: kernel arguments in device memory, no scratch reclaim
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
REPS=3 bash scripts/ab_env.sh base HIP_FORCE_DEV_KERNARG=1 HSA_NO_SCRATCH_RECLAIM=1 || exit 1
