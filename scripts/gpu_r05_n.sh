#!/bin/bash
# SRA standalone: the short-sequence kernels at larger N (CMX_SRA_SMALL_N) vs default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for n in 2048 5000 20000; do
  echo "== CMX_SRA_SMALL_N=$n"
  CMX_SRA_SMALL_N=$n timeout -k 10 120 python3 scripts/bench_sra.py || exit 1
done
