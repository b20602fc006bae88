#!/bin/bash
# One bench line + a rocprofv3 kernel trace of a short bench run (per-step census computed on
# the workstation with scripts/step_census.py).  Usage: bash scripts/quick_prof.sh TAG [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cut -c1-330 gpurun_out/bench_$TAG.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
