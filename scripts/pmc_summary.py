"""Per-kernel PMC summary of rocprofv3 --pmc runs (rocpd SQLite), with the gfx950 HBM-byte
correction of MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reports half the bytes of wide
coalesced streaming reads (double it); WRITE_SIZE (KB) is exact for 16-B stores.

Usage: python scripts/pmc_summary.py out.json fetch_run.db write_run.db WORKLOAD [kernel-substring ...]
Writes {"workload": WORKLOAD, "kernels": {name: {"launches", "FETCH_SIZE_kb", "WRITE_SIZE_kb",
"hbm_bytes_per_launch"}}}; roofline.py only reuses the bytes for the same workload tag
(bench.py's config.workload, e.g. "CMX-B2 train step 480x640 bs=2 K=40")."""
import json
import sqlite3
import sys


def per_kernel(db, counter):
    """{(kernel_name, dispatch_id): value} from rocpd's counters_collection view."""
    c = sqlite3.connect(db)
    rows = c.execute("select kernel_name, dispatch_id, value from counters_collection where counter_name = ?",
                     (counter,)).fetchall()
    out = {}
    for kname, disp, val in rows:
        out[(kname, disp)] = out.get((kname, disp), 0.0) + float(val)
    return out, None


def main():
    out_path, fdb, wdb, workload = sys.argv[1:5]
    wanted = sys.argv[5:]
    f, cols = per_kernel(fdb, "FETCH_SIZE")
    w, _ = per_kernel(wdb, "WRITE_SIZE")
    agg = {}
    for src, key in ((f, "FETCH_SIZE_kb"), (w, "WRITE_SIZE_kb")):
        for (kname, _), v in src.items():
            short = kname.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0].split("<")[0].split("::")[-1]
            if wanted and not any(s in kname for s in wanted):
                continue
            a = agg.setdefault(short, {"launches_fetch": 0, "launches_write": 0, "FETCH_SIZE_kb": 0.0, "WRITE_SIZE_kb": 0.0})
            a[key] += v
            a["launches_fetch" if key.startswith("FETCH") else "launches_write"] += 1
    res = {}
    for k, a in agg.items():
        nf, nw = max(1, a["launches_fetch"]), max(1, a["launches_write"])
        fetch = a["FETCH_SIZE_kb"] / nf * 1024.0
        write = a["WRITE_SIZE_kb"] / nw * 1024.0
        res[k] = {"launches": a["launches_fetch"], "FETCH_SIZE_kb_per_launch": fetch / 1024.0,
                  "WRITE_SIZE_kb_per_launch": write / 1024.0,
                  "hbm_bytes_per_launch": 2.0 * fetch + write}
    json.dump({"workload": workload, "correction": "hbm_bytes = 2 * FETCH_SIZE + WRITE_SIZE (gfx950, MI355X_MICROARCH.md HBM)",
               "kernels": res}, open(out_path, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
