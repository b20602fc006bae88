"""Ordered kernel timeline of one steady-state step from a rocprofv3 kernel trace of bench.py (the
step of median wall time, as scripts/step_census.py picks it): start offset, duration and queue of
every launch, so a stretch of the step (a stage's forward, its backward) can be read and summed.
Usage: python scripts/step_timeline.py <run_results.db> [from_us to_us]"""
import re
import sqlite3
import sys


def kname(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", n)


c = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
qcol = "queue_id" if "queue_id" in cols else ("stream_id" if "stream_id" in cols else None)
rows = c.execute(f"select start, end, name{', ' + qcol if qcol else ''} from kernels order by start").fetchall()
idx = [i for i, r in enumerate(rows) if kname(r[2]).startswith("step_masks")]


def wall(j):
    seg_ = rows[idx[j]:idx[j + 1]]
    return max(r[1] for r in seg_) - seg_[0][0]


walls = [(wall(j), j) for j in range(3, len(idx) - 2)] or [(0, len(idx) - 2)]
pick = sorted(walls)[len(walls) // 2][1]
seg = rows[idx[pick]:idx[pick + 1]]
t0 = seg[0][0]
lo = float(sys.argv[2]) if len(sys.argv) > 3 else -1
hi = float(sys.argv[3]) if len(sys.argv) > 3 else 1e12
print(f"step {pick}: {len(seg)} launches, wall {(max(r[1] for r in seg) - t0) / 1e3:.0f} us")
for r in seg:
    a, b = (r[0] - t0) / 1e3, (r[1] - t0) / 1e3
    if lo <= a <= hi:
        q = f" q{r[3]}" if qcol else ""
        print(f"{a:8.1f} {b - a:7.1f}{q}  {kname(r[2])[:90]}")
