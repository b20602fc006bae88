#!/bin/bash
# Bench sweep over one environment knob: VAR="CMX_X" VALUES="a b c" bash scripts/env_sweep.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in $VALUES; do
  env $VAR=$v timeout -k 10 100 python -u bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$VAR', '$v', d['value'], d['ms_per_step'])" || exit 1
done
