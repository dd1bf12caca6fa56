#!/bin/bash
# Round-3 A/B (on the GPU box via gpurun): the few-streams regime (tools/ab_solo.py)
# and the bench batch (tools/ab.py) for each library in $LIBS.
#   LIBS="lzma-java_amd/build/base/liblzma_mi355x.so lzma-java_amd/build/liblzma_mi355x.so" bash tools/ab_r03.sh [solo] [batch]
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
what=${*:-solo batch}
for w in $what; do
  for L in $LIBS; do
    case $w in
      solo) LZMA_AMD_LIB=$R/$L timeout -k 10 300 python3 $R/tools/ab_solo.py ${SOLO_ARGS:-} >> $O/solo.jsonl 2> $O/solo_err.log || { echo "solo $L failed rc=$?"; tail -5 $O/solo_err.log; exit 1; } ;;
      batch) LZMA_AMD_LIB=$R/$L timeout -k 10 200 python3 $R/tools/ab.py ${AB_ARGS:-} >> $O/ab.jsonl 2> $O/ab_err.log || { echo "ab $L failed rc=$?"; tail -5 $O/ab_err.log; exit 1; } ;;
    esac
  done
done
cat $O/solo.jsonl $O/ab.jsonl 2>/dev/null || true
