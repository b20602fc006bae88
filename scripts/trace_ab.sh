#!/bin/bash
# Kernel-traced bench per environment arm: the step census of each arm (scripts/step_census.py,
# 80 kernels) goes to gpurun_out/tab_TAG_<i>.census; the trace database itself only for the arms
# listed in KEEP (space-separated indices; each is ~15 MB and gpurun copies back <= 64 MiB):
#   KEEP="0" bash scripts/trace_ab.sh TAG base "CMX_FFM_STREAM=0"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
i=0
for arm in "$@"; do
  envs=""; [ "$arm" != "base" ] && envs="$arm"
  d=gpurun_out/tab_${TAG}_$i
  env $envs CMX_BENCH_NO_ROOFLINE=1 timeout -k 10 200 rocprofv3 --kernel-trace -d $d -o run -- python3 bench.py \
    --steps 12 --warmup 3 --no-cpu-baseline > $d.log 2>&1 || { echo "arm '$arm' failed"; tail -5 $d.log; exit 1; }
  db=$(ls $d/run_results.db $d/*/run_results.db 2>/dev/null | head -1)
  python3 scripts/step_census.py $db 80 > $d.census
  echo "[$i: $arm] $(sed -n 1,3p $d.census)"
  grep -o '"value": [0-9.]*' $d.log | head -1
  case " ${KEEP:-} " in *" $i "*) ;; *) rm -rf $d ;; esac
  i=$((i + 1))
done
