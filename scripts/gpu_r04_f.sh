#!/bin/bash
# host cost of a graph replay under HIP runtime launch options (bench lines with the idle-queue
# host enqueue time), interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/graph_env_r04_f.txt
: > $OUT
for r in 1 2; do
  for arm in base DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 HIP_FORCE_DEV_KERNARG=1; do
    envs=""; [ "$arm" != "base" ] && envs="$arm"
    out=$(env $envs timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null) || { echo "arm $arm failed" >> $OUT; exit 1; }
    echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['replay_ms']; print('rep $r', '[$arm]', d['value'], d['ms_per_step'], 'host', r['host_enqueue_idle_queue'], 'timed', r['timed'])" >> $OUT
  done
done
cat $OUT
