#!/bin/bash
# Round 6: the walk's solo time (full encodes, HIP events) for library variants, TEXT and BENCH.
# LIBS: library paths relative to the repo ("base" = the product build); build them first.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06/walk_ab
mkdir -p $O
cd $R
for L in ${LIBS:-base}; do
  if [ "$L" = base ]; then LP=$R/lzma-java_amd/build/liblzma_mi355x.so; else LP=$R/$L; fi
  for D in ${DATA:-text bench}; do
    WALK_FULL_ONLY=1 LZMA_AMD_LIB=$LP timeout -k 10 200 python3 -u tools/r06/walk_split.py $D > $O/one.txt 2>&1 || { echo "walk_split $L $D failed"; tail -5 $O/one.txt; exit 1; }
    echo "$L $D $(grep '^all' $O/one.txt)"
  done
done
