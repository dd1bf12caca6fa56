#!/bin/bash
# Round-3 walk scheduling: mf_walk time with the long-chains-first threshold
# LZG_WALK_LONG (4294967295 = off: stream order only), TEXT and BENCH; then the
# bench A/B with parity at the default threshold.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/wl; mkdir -p $O
for k in text bench; do
  for L in 4294967295 1024 512 256 128 64; do
    LZG_WALK_LONG=$L timeout -k 10 300 python3 $R/tools/walk_split.py $k | sed "s/}/, \"walk_long\": $L}/" >> $O/wl.jsonl 2>>$O/err.log || exit 1
  done
done
cat $O/wl.jsonl
