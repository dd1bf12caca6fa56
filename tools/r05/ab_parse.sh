#!/bin/bash
# Round 5 parse-kernel A/B: for each library (relative to the repo root), interleaved over
# ROUNDS rounds: one 4 MiB stream and the 512 / 4096 x 256 KiB batches (tools/ab_solo.py:
# parse HIP-event time, cycles per byte, first stream vs the oracle). One JSON line per row
# appended to gpurun_out/r05/$TAG/ab.jsonl; every run has its own time limit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05/${TAG:-ab}
mkdir -p $O
ROUNDS=${ROUNDS:-2}
for r in $(seq $ROUNDS); do
  for L in $LIBS; do
    LZMA_AMD_LIB=$R/$L timeout -k 10 180 python3 $R/tools/ab_solo.py --single ${SINGLE:-4194304} --shares ${SHARES:-512,4096} >> $O/ab.jsonl 2>> $O/ab.err || { echo "ab $L failed rc=$?"; exit 1; }
  done
done
python3 - $O/ab.jsonl <<'PY'
import json, sys, collections
rows = [json.loads(l) for l in open(sys.argv[1])]
agg = collections.defaultdict(list)
for r in rows:
    agg[(r["lib"].split("/build/")[-1], r["row"], r["streams"])].append((r["parse_ms"], r["parse_cycles_per_byte_per_stream"], r.get("first_stream_equals_oracle")))
for k, v in sorted(agg.items()):
    print(k, " ".join("%.1fms/%.0fcpb/%s" % x for x in v))
PY
