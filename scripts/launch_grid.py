"""Per-launch durations and grid shapes of one step (rocprofv3 kernel trace of bench.py),
filtered by kernel-name substrings.  Usage: python scripts/launch_grid.py <db> sub1 [sub2 ...]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
subs = sys.argv[2:]
rows = c.execute("select start, end, name, grid_x, grid_y, grid_z, workgroup_x, lds_size, vgpr_count "
                 "from kernels order by start").fetchall()
idx = [i for i, r in enumerate(rows) if r[2].startswith("adamw")]
seg = rows[idx[-2] + 1:idx[-1] + 1]
t0 = seg[0][0]
for s, e, n, gx, gy, gz, wx, lds, vg in seg:
    if not subs or any(k in n for k in subs):
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.2f}  blocks {gx // wx}x{gy}x{gz}  lds {lds:6d} vgpr {vg:3d}  {n[:70]}")
