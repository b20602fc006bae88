"""Summarise a rocprofv3 SQLite (rocpd) kernel trace: per-kernel totals per step.
Usage: python scripts/prof_summary.py <run_results.db> [steps] [out.txt]"""
import sqlite3
import sys


def main():
    db, steps = sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    out = open(sys.argv[3], "w") if len(sys.argv) > 3 else sys.stdout
    c = sqlite3.connect(db)
    rows = c.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
    tot = sum(r[2] for r in rows)
    print(f"# rocprofv3 --kernel-trace --stats summary of {db}", file=out)
    print(f"# total kernel time {tot / 1e3:.2f} ms over {steps:g} steps = {tot / 1e3 / steps:.3f} ms/step (durations in us)", file=out)
    print(f"{'calls/step':>10} {'us/step':>9} {'avg_us':>8} {'pct':>6}  kernel", file=out)
    for name, calls, dur, avg, pct in rows:
        print(f"{calls / steps:10.1f} {dur / steps:9.1f} {avg:8.2f} {pct:6.2f}  {name[:150]}", file=out)


if __name__ == "__main__":
    main()
