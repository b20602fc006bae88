"""Per-kernel SQ counter summary of a rocprofv3 --pmc run (rocpd SQLite): sums per kernel name
over its dispatches, and the wave-cycle split of MI355X_MICROARCH.md (SQ_WAIT_ANY = parked on
s_waitcnt / barrier, SQ_WAIT_INST_ANY = issue stall, SQ_ACTIVE_INST_ANY = issuing; quad-cycles).
Usage: python scripts/sq_summary.py run.db [kernel-substring]"""
import collections
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else None
rows = c.execute("select kernel_name, dispatch_id, counter_name, value from counters_collection").fetchall()
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for k, d, n, v in rows:
    k = k.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    if flt and flt not in k:
        continue
    agg[k][n] += float(v)
    disp[k].add(d)
for k, cs in agg.items():
    nd = len(disp[k])
    print(f"{k[:70]}  dispatches {nd}")
    for n in sorted(cs):
        print(f"    {n:28s} {cs[n] / nd:14.1f} per dispatch")
    wc = cs.get("SQ_WAVE_CYCLES", 0.0)
    if wc:
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if n in cs:
                print(f"    {n + ' / WAVE_CYCLES':40s} {cs[n] / wc:6.3f}")
