"""Reduce rocprofv3 CSV outputs for profiles/ (see tools/profile_round.sh).

stats   <dir> <out.csv>: per-kernel calls / total / mean duration (ms) with the
        dispatch's grid, LDS, VGPR and SGPR, from the kernel trace.
counters <dir> <out.json> [workload-json]: per-kernel sum of every collected counter
        per launch (e.g. the SQ_INSTS_* issue counters behind bench.py's roofline.issue).
traffic <fetch_dir> <write_dir> <out.json>: per-kernel FETCH_SIZE and WRITE_SIZE
        per launch in bytes. rocprofv3 reports both in KiB; on gfx950 FETCH_SIZE
        counts 64 B per memory-side read request while wide streaming reads
        move 128 B per request (MI355X_MICROARCH.md, HBM section), so the
        corrected read bytes are 2 x FETCH_SIZE for such reads. The kernels
        here mostly make narrow scattered accesses, for which the guide gives no
        calibration: both the raw and the doubled figure are recorded.
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def short(name):
    name = re.sub(r"\(.*", "", name).replace("void ", "").strip()
    if "rocprim" in name:
        m = re.search(r"detail::(radix_sort_onesweep_\w+|partition_impl|\w+_kernel)", name)
        return "rocprim::" + (m.group(1) if m else "kernel")
    return re.sub(r"^lzg::", "", name)


def rows(d, suffix):
    out = []
    for f in glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def stats(d, out):
    agg = collections.OrderedDict()
    for r in rows(d, "kernel_trace.csv"):
        k = short(r["Kernel_Name"])
        a = agg.setdefault(k, {"calls": 0, "ns": 0, "grid": r.get("Grid_Size_X", r.get("Grid_Size", "")),
                               "lds": r.get("LDS_Block_Size", r.get("Group_Segment_Size", "")),
                               "vgpr": r.get("Arch_VGPR_Count", r.get("VGPR_Count", "")),
                               "sgpr": r.get("SGPR_Count", "")})
        a["calls"] += 1
        a["ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot = sum(a["ns"] for a in agg.values()) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_ms", "avg_ms", "pct", "grid_x", "lds_bytes", "vgpr", "sgpr"])
        for k, a in sorted(agg.items(), key=lambda kv: -kv[1]["ns"]):
            w.writerow([k, a["calls"], "%.3f" % (a["ns"] / 1e6), "%.3f" % (a["ns"] / 1e6 / a["calls"]),
                        "%.2f" % (100.0 * a["ns"] / tot), a["grid"], a["lds"], a["vgpr"], a["sgpr"]])
    print(open(out).read())


def traffic(fd, wd, out, workload=None):
    res = {}
    for d, cname in ((fd, "FETCH_SIZE"), (wd, "WRITE_SIZE")):
        per = collections.defaultdict(float)
        disp = collections.defaultdict(set)
        for r in rows(d, "counter_collection.csv"):
            if r["Counter_Name"] != cname:
                continue
            k = short(r["Kernel_Name"])
            per[k] += float(r["Counter_Value"]) * 1024.0
            disp[k].add(r["Dispatch_Id"])
        for k, v in per.items():
            e = res.setdefault(k, {})
            e[cname.lower() + "_bytes_per_launch"] = v / max(len(disp[k]), 1)
            e["launches"] = len(disp[k])
    for k, e in res.items():
        if k.startswith("_"):
            continue
        f = e.get("fetch_size_bytes_per_launch", 0.0)
        w = e.get("write_size_bytes_per_launch", 0.0)
        e["traffic_bytes_per_launch_raw"] = f + w
        e["traffic_bytes_per_launch"] = 2 * f + w
    res["_workload"] = json.loads(workload) if workload else {
        "bytes_per_gpu": 1 << 30, "chunk": 256 << 10, "data": "bench", "dict_log": 26,
        "command": "bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-verify"}
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


def counters(d, out, workload=None):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in rows(d, "counter_collection.csv"):
        k = short(r["Kernel_Name"])
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    res = {k: dict({c: v / max(len(disp[k]), 1) for c, v in cs.items()}, launches=len(disp[k]))
           for k, cs in per.items()}
    res["_workload"] = json.loads(workload) if workload else {}
    res["_cus"] = 256
    res["_sclk_hz"] = 2.4e9
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    if sys.argv[1] == "stats":
        stats(sys.argv[2], sys.argv[3])
    elif sys.argv[1] == "counters":
        counters(sys.argv[2], sys.argv[3], sys.argv[4] if len(sys.argv) > 4 else None)
    else:
        traffic(sys.argv[2], sys.argv[3], sys.argv[4], sys.argv[5] if len(sys.argv) > 5 else None)
