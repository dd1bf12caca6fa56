"""Summarise a rocprofv3 --kernel-trace --stats database (rocpd SQLite) as CSV.

usage: python tools/rocprof_summary.py <run_results.db> <out.csv> [title]
Columns: kernel (short name), calls, total_ms, avg_ms, pct, grid (threads), lds_bytes,
vgpr, sgpr, scratch as rocprofv3 records them.  Durations come from the database's top_kernels view
(microseconds in the rocpd schema of ROCm 7.2: checked against the HIP-event
times bench.py reports for the same kernels).
"""
import csv
import re
import sqlite3
import sys


def short(name: str) -> str:
    if "rocprim" in name:
        m = re.search(r"detail::(radix_sort_onesweep_\w+|partition_impl|\w+_kernel)", name)
        return "rocprim::" + (m.group(1) if m else "kernel")
    name = re.sub(r"\(.*", "", name)          # drop the argument list
    return name.replace("void ", "").strip()


def main():
    db, out = sys.argv[1], sys.argv[2]
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    meta = {}
    for name, grid, lds, vgpr, sgpr, scr in c.execute(
            "select name, max(grid_x), max(lds_size), max(vgpr_count), max(sgpr_count), max(scratch_size) "
            "from kernels group by name"):
        meta[name] = (grid, lds, vgpr, sgpr, scr)
    merged = {}
    for name, calls, total, avg, pct in rows:
        k = short(name)
        g = meta.get(name, (None,) * 5)
        if k in merged:
            m = merged[k]
            m[0] += calls; m[1] += total; m[3] += pct
            m[2] = m[1] / m[0]
        else:
            merged[k] = [calls, total, avg, pct, *g]
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_ms", "avg_ms", "pct", "grid_x", "lds_bytes", "vgpr", "sgpr",
                    "scratch"])
        for k, m in sorted(merged.items(), key=lambda kv: -kv[1][1]):
            w.writerow([k, m[0], "%.3f" % (m[1] / 1e3), "%.3f" % (m[2] / 1e3), "%.2f" % m[3], *m[4:]])
    print(open(out).read())


if __name__ == "__main__":
    main()
