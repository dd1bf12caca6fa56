#!/bin/bash
# A/B of library builds on the bench workload (on the GPU box via gpurun):
#   LIBS="lzma-java_amd/build/liblzma_mi355x.so lzma-java_amd/build/v1/liblzma_mi355x.so" bash tools/ab.sh
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab
mkdir -p $O
for L in $LIBS; do
  LZMA_AMD_LIB=$R/$L timeout -k 10 200 python3 $R/tools/ab.py ${AB_ARGS:-} >> $O/ab.jsonl 2> $O/ab_err.log || { echo "ab $L failed rc=$?"; tail -5 $O/ab_err.log; exit 1; }
  tail -1 $O/ab.jsonl
done
