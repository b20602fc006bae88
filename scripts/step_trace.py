"""Launch-by-launch trace of one step from a rocprofv3 kernel trace of bench.py (the launches
between the last two AdamW launches), with start offset, duration and gap to the previous end.
Usage: python scripts/step_trace.py <run_results.db> [filter-substring]"""
import re
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else None
rows = c.execute("select start, end, name from kernels order by start").fetchall()
idx = [i for i, r in enumerate(rows) if r[2].replace("void ", "").startswith("adamw")]
seg = rows[idx[-2] + 1:idx[-1] + 1]
t0 = seg[0][0]
prev_end = t0
for s, e, n in seg:
    k = re.sub(r"\(.*", "", n.replace("void ", "").replace("(anonymous namespace)::", ""))[:90]
    if flt is None or flt in k:
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.2f} {(s - prev_end) / 1e3:7.2f}  {k}")
    prev_end = max(prev_end, e)
