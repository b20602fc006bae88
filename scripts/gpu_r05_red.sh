#!/bin/bash
# SRA dK/dV slab reduce with all of a thread's chunk loads in flight: tests + standalone
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "sra" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r05_red.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r05_red.log; grep -E "^FAILED" gpurun_out/pytest_r05_red.log | head -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 scripts/bench_sra.py || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/red_prof -o run -- python3 scripts/bench_sra.py > gpurun_out/red_prof.log 2>&1 || exit 1
grep -h "sra_dkv_reduce\|sra_dkv_fast\|sra_dq_fast" $(find gpurun_out/red_prof -name "*kernel_stats.csv") | cut -d, -f1-5 | head -8
rm -rf gpurun_out/red_prof
