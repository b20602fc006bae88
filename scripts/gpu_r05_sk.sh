#!/bin/bash
# streaming GEMM grid: the largest K it takes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/gemm_census.py --ab GEMM_STREAM_K=128,256,512 2>/dev/null | head -16
