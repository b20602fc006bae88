#!/bin/bash
# 64 x 128 tiles for problems just over one round of 64 x 64 blocks (CMX_GEMM_MID): tests + census
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CMX_GEMM_MID=50 timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -2
timeout -k 10 300 python3 scripts/gemm_census.py --ab GEMM_MID=0,25,50,100 2>/dev/null | head -14
