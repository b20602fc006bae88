"""Per-step kernel census from a rocprofv3 kernel trace of bench.py: the launches between the
last two AdamW launches (one HIP-graph replay = one step), grouped by kernel family.
Usage: python scripts/step_census.py <run_results.db> [top]"""
import collections
import re
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = c.execute("select start, end, name from kernels order by start").fetchall()
idx = [i for i, r in enumerate(rows) if r[2].replace("void ", "").startswith("adamw")]
seg = rows[idx[-2] + 1:idx[-1] + 1]
print(f"launches/step {len(seg)}  wall {(seg[-1][1] - seg[0][0]) / 1e3:.0f} us  busy {sum(r[1] - r[0] for r in seg) / 1e3:.0f} us")
cat = collections.defaultdict(lambda: [0, 0.0])
for s, e, n in seg:
    k = re.sub(r"\(.*", "", n.replace("void ", "").replace("(anonymous namespace)::", ""))
    cat[k][0] += 1
    cat[k][1] += (e - s) / 1e3
for k, (n, t) in sorted(cat.items(), key=lambda x: -x[1][1])[:top]:
    print(f"{n:5d} {t:8.1f} {t / n:7.2f}  {k[:100]}")
