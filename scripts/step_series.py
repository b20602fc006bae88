"""Per-step series from a rocprofv3 kernel trace of bench.py: for every step (the launches
after one AdamW up to and including the next), its wall and busy time, and the per-kernel
duration ratio between the first and the last few steps -- tells a uniform slow-down
(clock / power state) from a family-specific one (first touch, allocator growth).
Usage: python scripts/step_series.py <run_results.db> [n_compare]"""
import collections
import re
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
ncmp = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows = c.execute("select start, end, name from kernels order by start").fetchall()
idx = [i for i, r in enumerate(rows) if r[2].replace("void ", "").startswith("adamw")]
steps = [rows[a + 1:b + 1] for a, b in zip(idx, idx[1:])]
t_first = rows[0][0]
print(f"{len(rows)} launches, {len(idx)} AdamW launches, {len(steps)} whole steps")
for i, seg in enumerate(steps):
    wall = (seg[-1][1] - seg[0][0]) / 1e3
    busy = sum(r[1] - r[0] for r in seg) / 1e3
    print(f"step {i:3d} at {(seg[0][0] - t_first) / 1e6:8.1f} ms  launches {len(seg):4d}  wall {wall:8.0f} us  busy {busy:8.0f} us")


def fam(seg):
    d = collections.defaultdict(float)
    for s, e, n in seg:
        d[re.sub(r"\(.*", "", n.replace("void ", "").replace("(anonymous namespace)::", ""))[:60]] += (e - s) / 1e3
    return d


if len(steps) >= 2 * ncmp:
    a, b = collections.defaultdict(float), collections.defaultdict(float)
    for seg in steps[:ncmp]:
        for k, v in fam(seg).items():
            a[k] += v / ncmp
    for seg in steps[-ncmp:]:
        for k, v in fam(seg).items():
            b[k] += v / ncmp
    print(f"\nper-kernel us/step, first {ncmp} vs last {ncmp} steps (sorted by the difference)")
    for k in sorted(a, key=lambda k: -(a[k] - b.get(k, 0.0)))[:40]:
        print(f"{a[k]:9.1f} {b.get(k, 0.0):9.1f}  x{a[k] / max(b.get(k, 1e-9), 1e-9):5.2f}  {k}")
