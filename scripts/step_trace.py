"""Launch-by-launch trace of one step from a rocprofv3 kernel trace of bench.py: the steady-state
replay of median wall time (as scripts/step_census.py picks it), with start offset, duration, the
gap to the latest end so far (negative: overlaps a launch still running on another stream) and
the queue the launch came from.
Usage: python scripts/step_trace.py <run_results.db> [filter-substring] [--gaps MIN_US]"""
import re
import sqlite3
import sys


def kname(n):
    """as scripts/step_census.py: no 'void ', no '(anonymous namespace)::', no argument list"""
    return re.sub(r"\(.*", "", n.replace("void ", "").replace("(anonymous namespace)::", ""))


args = [a for a in sys.argv[1:]]
gmin = None
if "--gaps" in args:
    i = args.index("--gaps")
    gmin = float(args[i + 1])
    del args[i:i + 2]
c = sqlite3.connect(args[0])
flt = args[1] if len(args) > 1 else None
cols = [r[1] for r in c.execute("pragma table_info(kernels)").fetchall()]
qcol = "queue_id" if "queue_id" in cols else ("stream_id" if "stream_id" in cols else None)
rows = c.execute(f"select start, end, name{', ' + qcol if qcol else ''} from kernels order by start").fetchall()
idx = [i for i, r in enumerate(rows) if kname(r[2]).startswith("step_masks")]
if len(idx) < 3:
    idx = [i + 1 for i, r in enumerate(rows) if kname(r[2]).startswith("adamw")]
walls = [(max(r[1] for r in rows[idx[j]:idx[j + 1]]) - rows[idx[j]][0], j) for j in range(3, len(idx) - 2)] \
    or [(0, len(idx) - 2)]
pick = sorted(walls)[len(walls) // 2][1]
seg = rows[idx[pick]:idx[pick + 1]]
t0 = seg[0][0]
prev_end = t0
for r in seg:
    s, e, n = r[0], r[1], r[2]
    q = r[3] if qcol else ""
    k = kname(n)[:90]
    gap = (s - prev_end) / 1e3
    if (flt is None or flt in k) and (gmin is None or gap >= gmin):
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.2f} {gap:7.2f} q{q}  {k}")
    prev_end = max(prev_end, e)
