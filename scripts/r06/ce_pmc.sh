#!/bin/bash
# round-6: CE kernels standalone (scripts/bench_ops.py ce) -- timings, then two SQ counter passes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 120 python3 scripts/bench_ops.py ce > gpurun_out/r06/ce_ops.txt 2>&1
rc=$?; echo "ops rc=$rc"; cat gpurun_out/r06/ce_ops.txt; [ $rc -eq 0 ] || exit $rc
i=0
for CT in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
          "SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $CT --kernel-include-regex "ce_" -d gpurun_out/r06/ce_pmc$i -o run -- python3 scripts/bench_ops.py ce > gpurun_out/r06/ce_pmc$i.log 2>&1
  rc=$?; echo "pmc$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  db=$(ls gpurun_out/r06/ce_pmc$i/*.db gpurun_out/r06/ce_pmc$i/*/*.db 2>/dev/null | head -1)
  python3 - "$db" <<'PY'
import collections, sqlite3, sys
c = sqlite3.connect(sys.argv[1])
agg = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(set)
for d, k, cn, v in c.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection"):
    n = k.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:40]
    agg[n][cn] += v; disp[n].add(d)
for n, a in agg.items():
    nd = len(disp[n]); w = max(a.get("SQ_WAVES", 1), 1)
    print(n, nd, "per-wave:", {k: round(v / w, 1) for k, v in sorted(a.items())})
PY
  rm -rf gpurun_out/r06/ce_pmc$i
done
