#!/bin/bash
# Round 6: where one stream's parse spends its wave cycles (SQ counters, one --pmc pass of 8
# SQ counters) -- one 4 MiB BENCH stream (tools/enc_scaling.py), the product library.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06/${TAG:-single_pmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH --output-format csv -d /tmp/sp -o run -- python3 $R/tools/enc_scaling.py ${BYTES:-4194304} 1 bench > $O/pmc.log 2>&1 || { echo "pmc failed rc=$?"; tail -5 $O/pmc.log; exit 1; }
f=$(find /tmp/sp -name "*counter_collection.csv" | head -1)
cp $f $O/counters.csv
python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "enc_kernel" in r.get("Kernel_Name", ""):
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(acc):
    print("%-22s %16.0f" % (k, acc[k]))
PY
