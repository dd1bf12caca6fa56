"""Fold a rocprofv3 CSV output directory into a per-kernel summary (stdout).

Kernel trace: calls and mean/total duration per kernel. Counter collection:
per-kernel sum of each counter over its dispatches, and the sum divided by
the number of dispatches.
"""
import collections
import csv
import glob
import os
import re
import sys


def short(name):
    name = re.sub(r"\(.*", "", name).replace("void ", "").strip()
    if "rocprim" in name:
        return "rocprim"
    return name[:60]


def main(d):
    files = glob.glob(os.path.join(d, "**", "*.csv"), recursive=True)
    for f in sorted(files):
        base = os.path.basename(f)
        rows = list(csv.DictReader(open(f)))
        if not rows:
            continue
        if base.endswith("kernel_trace.csv"):
            agg = collections.defaultdict(lambda: [0, 0.0])
            for r in rows:
                k = short(r["Kernel_Name"])
                agg[k][0] += 1
                agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            print("# kernel trace: kernel, calls, total_ms, avg_ms")
            for k, (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
                print("%s,%d,%.3f,%.3f" % (k, n, ms, ms / n))
        elif base.endswith("counter_collection.csv"):
            agg = collections.defaultdict(float)
            disp = collections.defaultdict(set)
            for r in rows:
                k = short(r["Kernel_Name"])
                agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
                disp[k].add(r["Dispatch_Id"])
            print("# counters: kernel, counter, sum, per_dispatch, dispatches")
            for (k, c), v in sorted(agg.items()):
                n = len(disp[k])
                print("%s,%s,%.6g,%.6g,%d" % (k, c, v, v / n, n))
        elif base.endswith("stats.csv"):
            print("# %s" % base)
            print(open(f).read())


if __name__ == "__main__":
    main(sys.argv[1])
