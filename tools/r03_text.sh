#!/bin/bash
# Round-3 TEXT vs BENCH phase profile (LZG_PROF build) and the strong-scaling projection
# (on the GPU box via gpurun); each GPU step has its own limit.
#   usage: tools/r03_text.sh [phase] [strong]
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
fail() { echo "$1 failed rc=$2"; exit $2; }
for s in ${*:-phase strong}; do
  case $s in
    phase)
      for k in text bench; do
        LZMA_AMD_LIB=$R/lzma-java_amd/build/prof/liblzma_mi355x.so timeout -k 10 300 \
          python3 $R/tools/enc_scaling.py 262144 1024 $k > $O/phase_$k.txt 2>&1 || fail phase_$k $?
      done
      tail -n 40 $O/phase_text.txt $O/phase_bench.txt ;;
    strong)
      timeout -k 10 400 python3 $R/tools/strong_share.py --steps 2 > $O/strong_share.jsonl 2> $O/strong_err.log || fail strong $?
      cat $O/strong_share.jsonl ;;
  esac
done
