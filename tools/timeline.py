"""Timeline of a bench run from a rocprofv3 kernel trace: per kernel launch its start and
end relative to the first launch, the queue it ran on, and for the last --steps steps the
GPU-idle gaps (no kernel running on any queue) and the busy time per kernel.

usage: python tools/timeline.py <rocprofv3 -d dir> [--from-kernel enc_kernel] [--last N]
"""
import argparse
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from round_reduce import short  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=120, help="print the last N launches")
    ap.add_argument("--window", type=int, default=2, help="gap analysis over the last W parse launches' steps")
    args = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(args.dir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                         r.get("Queue_Id", r.get("Stream_Id", "?"))))
    rows.sort()
    if not rows:
        print("no kernel trace rows")
        return
    t0 = rows[0][0]
    for s, e, k, q in rows[-args.last:]:
        print("%10.3f %10.3f %8.3f q%s %s" % ((s - t0) / 1e6, (e - t0) / 1e6, (e - s) / 1e6, q, k))
    # the window: from the start of the W-th last enc_kernel's step (its preceding mf_keys) to the end
    parses = [i for i, r in enumerate(rows) if r[2].startswith("enc_kernel")]
    keys = [i for i, r in enumerate(rows) if r[2].startswith("mf_keys")]
    if len(parses) < args.window or not keys:
        return
    first_parse = parses[-args.window]
    start_i = max([i for i in keys if i < first_parse] or [0])
    win = rows[start_i:]
    ws, we = win[0][0], max(r[1] for r in win)
    busy, gaps, cur_end = 0, [], ws
    for s, e, k, q in win:
        if s > cur_end:
            gaps.append((cur_end, s, k))
        cur_end = max(cur_end, e)
    span = we - ws
    idle = sum(b - a for a, b, _ in gaps)
    print("window %.3f ms over %d launches, GPU idle %.3f ms in %d gaps" % (span / 1e6, len(win), idle / 1e6, len(gaps)))
    for a, b, k in sorted(gaps, key=lambda g: g[0] - g[1])[:15]:
        print("  gap %8.3f ms at %10.3f before %s" % ((b - a) / 1e6, (a - t0) / 1e6, k))
    per = {}
    for s, e, k, q in win:
        per[k] = per.get(k, 0) + e - s
    for k, v in sorted(per.items(), key=lambda x: -x[1])[:20]:
        print("  %-40s %9.3f ms" % (k, v / 1e6))


if __name__ == "__main__":
    main()
