#!/bin/bash
# Round 6: the walk's waves per CU capped through dynamic LDS per wave (experiment build,
# LZG_WALK_LDS bytes per 64-lane block: 160 KiB / bytes blocks per CU), solo walk times of full
# encodes for TEXT and BENCH (tools/r06/walk_split.py, WALK_FULL_ONLY).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06/walk_lds
mkdir -p $O
cd $R
for L in ${LDS:-0 5120 10240 20480}; do
  for D in ${DATA:-text bench}; do
    LZG_WALK_LDS=$L WALK_FULL_ONLY=1 LZMA_AMD_LIB=$R/lzma-java_amd/build/exp/liblzma_mi355x.so timeout -k 10 200 python3 -u tools/r06/walk_split.py $D > $O/one.txt 2>&1 || { echo "walk_split $L $D failed"; tail -5 $O/one.txt; exit 1; }
    echo "lds $L $D $(grep '^all' $O/one.txt)"
  done
done
