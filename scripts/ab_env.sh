#!/bin/bash
# Interleaved A/B of environment settings on the bench: each argument is one setting
# ("CMX_A=1 CMX_B=2", or "base" for none), run REPS times round-robin so drift hits every arm.
#   REPS=2 bash scripts/ab_env.sh base "CMX_LN_NCH=5" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
# one throwaway run first: the first bench on a fresh box runs a few % slow (clocks / caches)
timeout -k 10 100 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > /dev/null 2>&1 || { echo "warm-up failed"; exit 1; }
for r in $(seq ${REPS:-2}); do
  for arm in "$@"; do
    envs=""; [ "$arm" != "base" ] && envs="$arm"
    out=$(env $envs timeout -k 10 100 python -u bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline 2>/dev/null) || { echo "arm '$arm' failed"; exit 1; }
    echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; print('rep $r', '[$arm]', d['value'], d['ms_per_step'], 'gemm_family_us', r.get('total_us'), 'grouped_us', (r.get('second') or {}).get('avg_launch_us'))"
  done
done
