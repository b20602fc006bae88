"""Per-queue busy time of one step (between the last two AdamW launches) of a rocprofv3 kernel
trace, and how much of the step the main queue alone covers: the critical-path view of a step
whose FFM branch and weight gradients run on side streams.
Usage: python scripts/stream_census.py <run_results.db>"""
import collections
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select start, end, name, queue_id, stream_id from kernels order by start").fetchall()
idx = [i for i, r in enumerate(rows) if r[2].startswith("adamw")]
seg = rows[idx[-2] + 1:idx[-1] + 1]
t0, t1 = seg[0][0], seg[-1][1]
print(f"step wall {(t1 - t0) / 1e3:.0f} us, {len(seg)} launches")
by = collections.defaultdict(lambda: [0, 0.0])
for s, e, n, q, st in seg:
    by[(q, st)][0] += 1
    by[(q, st)][1] += (e - s) / 1e3
for k, (n, t) in sorted(by.items(), key=lambda kv: -kv[1][1]):
    print(f"queue {k[0]} stream {k[1]}: {n} launches, {t:.0f} us busy")
# union of busy intervals (any queue) and gaps
iv = sorted((s, e) for s, e, *_ in seg)
busy, cs, ce = 0, iv[0][0], iv[0][1]
for s, e in iv[1:]:
    if s > ce:
        busy += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
print(f"GPU busy (union over queues) {busy / 1e3:.0f} us, idle {(t1 - t0 - busy) / 1e3:.0f} us")
