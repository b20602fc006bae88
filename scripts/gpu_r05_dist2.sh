#!/bin/bash
# kernel traces of the one-GPU step with and without the data-parallel path (world size 1):
# where the DP machinery's per-step cost goes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
d=gpurun_out/dtr_plain
timeout -k 10 200 rocprofv3 --kernel-trace -d $d -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $d.log 2>&1 || exit 1
python3 scripts/step_census.py $(find $d -name "*.db" | head -1) 400 > gpurun_out/dist_census_plain.txt 2>&1
rm -rf $d
export WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29517 CMX_FORCE_DIST=1
d=gpurun_out/dtr_force
timeout -k 10 300 rocprofv3 --kernel-trace -d $d -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
python3 scripts/step_census.py $(find $d -name "*.db" | head -1) 400 > gpurun_out/dist_census_force.txt 2>&1
rm -rf $d
head -3 gpurun_out/dist_census_plain.txt | cut -c1-250
head -3 gpurun_out/dist_census_force.txt | cut -c1-250
tail -16 gpurun_out/dist_census_plain.txt
tail -16 gpurun_out/dist_census_force.txt
