#!/bin/bash
# round-6: kernel trace of the bench + step census + per-queue timeline (trace database comes back)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
CMX_BENCH_NO_ROOFLINE=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r06/trace_$1 -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r06/trace_$1.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
db=$(ls gpurun_out/r06/trace_$1/*.db gpurun_out/r06/trace_$1/*/*.db 2>/dev/null | head -1)
python3 scripts/step_census.py $db 80 > gpurun_out/r06/census_$1.txt 2>&1
python3 scripts/step_timeline.py $db > gpurun_out/r06/timeline_$1.txt 2>&1
head -3 gpurun_out/r06/census_$1.txt
