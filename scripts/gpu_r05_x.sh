#!/bin/bash
# two kernel-traced bench runs: the idle gaps over 20 us inside the median step, with neighbours
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  d=gpurun_out/gap_$rep
  timeout -k 10 200 rocprofv3 --kernel-trace -d $d -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $d.log 2>&1 || exit 1
  db=$(find $d -name "*.db" | head -1)
  python3 scripts/step_census.py $db 5 > gpurun_out/gaps_r05_x_$rep.txt 2>&1
  head -60 gpurun_out/gaps_r05_x_$rep.txt | grep -v "^ *[0-9]\+ \+[0-9.]\+ \+[0-9.]\+  "
  rm -rf $d
done
