#!/bin/bash
# SRA standalone per-kernel split (default small kernels vs the fast kernels at stages 3/4)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for arm in base CMX_SRA_SMALL_N=0; do
  envs=""; [ "$arm" != "base" ] && envs="$arm"
  d=gpurun_out/sra_$arm
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 scripts/bench_sra.py > $d.log 2>&1 || { echo "$arm failed"; tail $d.log; exit 1; }
  echo "== $arm"; cat $d.log
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in rows:
    if 'sra' in r['Name']: print('%8s %9.2f %s' % (r['Calls'], float(r['AverageNs'])/1e3, r['Name'][:70]))
"
done
