#!/bin/bash
# mf_walk time vs waves per CU (LZG_WALK_LDS: dynamic LDS per 64-lane block caps the blocks per CU)
R=$GRAFT_REPO_ROOT
for L in 0 8192 16384 32768; do
  LZG_WALK_LDS=$L timeout -k 10 200 python3 $R/tools/ab.py --reps 1 --parity 0 > /tmp/w.json 2>/dev/null || { echo "lds $L failed"; exit 1; }
  python3 -c "import json; d=json.load(open('/tmp/w.json')); print('walk_lds', $L, 'mf_walk', d['kernels_ms']['mf_walk'], 'MBps', round(d['MBps'],1))"
done
