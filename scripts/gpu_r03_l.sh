#!/bin/bash
# Standalone SRA (per stage) and DWConv timings at the B2 480x640 bs=2 shapes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_l}
timeout -k 10 200 python -u scripts/bench_sra.py > gpurun_out/sra_$TAG.txt 2>&1 || exit $?
timeout -k 10 200 python -u scripts/bench_sra.py sweep >> gpurun_out/sra_$TAG.txt 2>&1 || exit $?
cat gpurun_out/sra_$TAG.txt
timeout -k 10 200 python -u scripts/bench_dw.py > gpurun_out/dw_$TAG.txt 2>&1 || exit $?
cat gpurun_out/dw_$TAG.txt
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/sraprof_$TAG -o run -- python3 scripts/bench_sra.py > /dev/null 2>&1 || exit $?
db=$(ls gpurun_out/sraprof_$TAG/*.db gpurun_out/sraprof_$TAG/*/*.db 2>/dev/null | head -1)
python3 scripts/prof_summary.py $db > gpurun_out/sra_kernels_$TAG.txt 2>&1; head -30 gpurun_out/sra_kernels_$TAG.txt
rm -rf gpurun_out/sraprof_$TAG
