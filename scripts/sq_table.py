"""Per-kernel SQ counter table from a rocprofv3 --pmc run (rocpd SQLite): per dispatch averages,
and the wave-cycle split WAIT_ANY (parked on s_waitcnt / barrier) + WAIT_INST_ANY (issue
stalls) + ACTIVE_INST_ANY (issuing) ~= WAVE_CYCLES (MI355X_MICROARCH.md rocprofv3 PMC slots).
Usage: python scripts/sq_table.py run.db"""
import collections
import sqlite3
import sys


def main(db):
    c = sqlite3.connect(db)
    rows = c.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection").fetchall()
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for d, k, cn, v in rows:
        name = k.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:60]
        agg[name][cn] += v
        disp[name].add(d)
    print(f"{'kernel':60s} {'disp':>5s} {'waves':>7s} {'cyc/wave':>9s} {'wait%':>6s} {'stall%':>6s} {'active%':>7s} "
          f"{'VALU/w':>7s} {'LDS/w':>6s}")
    for name, a in sorted(agg.items(), key=lambda kv: -kv[1]["SQ_WAVE_CYCLES"]):
        n = len(disp[name])
        wc = a["SQ_WAVE_CYCLES"] or 1.0
        waves = a["SQ_WAVES"] / n
        print(f"{name:60s} {n:5d} {waves:7.0f} {4 * wc / max(a['SQ_WAVES'], 1):9.0f} "
              f"{100 * a['SQ_WAIT_ANY'] / wc:6.1f} {100 * a['SQ_WAIT_INST_ANY'] / wc:6.1f} "
              f"{100 * a['SQ_ACTIVE_INST_ANY'] / wc:7.1f} {a['SQ_INSTS_VALU'] / max(a['SQ_WAVES'], 1):7.0f} "
              f"{a['SQ_INSTS_LDS'] / max(a['SQ_WAVES'], 1):6.0f}")


if __name__ == "__main__":
    main(sys.argv[1])
