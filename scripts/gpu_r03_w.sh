#!/bin/bash
# Replay-boundary and in-step idle time from a kernel trace of the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_w}
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 10 --warmup 2 \
  --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || exit $?
db=$(ls gpurun_out/prof_$TAG/*.db gpurun_out/prof_$TAG/*/*.db 2>/dev/null | head -1)
python3 scripts/step_census.py $db 30 > gpurun_out/step_census_$TAG.txt 2>&1
head -4 gpurun_out/step_census_$TAG.txt
python3 - "$db" <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
rows = c.execute("select start, end, name from kernels order by start").fetchall()
idx = [i for i, r in enumerate(rows) if r[2].replace("void ", "").startswith("adamw")]
for a, b in zip(idx[-6:-1], idx[-5:]):
    print(f"step span {(rows[b][1] - rows[a][1]) / 1e3:.0f} us; boundary gap {(rows[a + 1][0] - rows[a][1]) / 1e3:.1f} us; "
          f"first {rows[a + 1][2][:40]}")
PY
rm -f $db
