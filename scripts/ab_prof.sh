#!/bin/bash
# Interleaved A/B of environment settings under a kernel trace: per arm and rep, the summed
# kernel time of the traced bench and the per-launch averages of the kernels matching REGEX.
#   REPS=2 bash scripts/ab_prof.sh 'dw2_|gemm_bf16' base "CMX_LIB_VARIANT=dwnt"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
RX=$1; shift
for rep in $(seq ${REPS:-2}); do
  for arm in "$@"; do
    envs=""; [ "$arm" != "base" ] && envs="$arm"
    d=gpurun_out/abp_$rep_$$
    env $envs timeout -k 10 200 rocprofv3 --kernel-trace -d $d -o run -- python3 bench.py --steps 10 --warmup 3 \
      --no-cpu-baseline > $d.log 2>&1 || { echo "arm '$arm' failed"; exit 1; }
    db=$(find $d -name "*.db" | head -1)
    echo "rep $rep [$arm] $(python3 scripts/step_census.py $db 400 | head -1)"
    python3 scripts/step_census.py $db 400 | grep -E "$RX" | head -12 | sed "s/^/    /"
    rm -rf $d $d.log
  done
done
