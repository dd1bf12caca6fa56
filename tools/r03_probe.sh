#!/bin/bash
# Round-3 probe (run on the GPU box via gpurun): host CPU share, strong-scaling
# shares, single-stream end-to-end time and its phase profile.
#   usage: tools/r03_probe.sh [cpu] [strong] [single] [phase]   (default: all)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
fail() { echo "$1 failed rc=$2"; exit $2; }
steps=${*:-cpu strong single phase}
for s in $steps; do
  case $s in
    cpu) timeout -k 10 300 python3 $R/tools/cpu_scaling.py > $O/cpu_scaling.jsonl 2> $O/cpu_scaling.err || fail cpu $?
         cat $O/cpu_scaling.jsonl ;;
    strong) timeout -k 10 300 python3 $R/tools/strong_share.py > $O/strong_share.jsonl 2> $O/strong_share.err || fail strong $?
            cat $O/strong_share.jsonl ;;
    single) timeout -k 10 300 python3 $R/tools/chunk_sweep.py --data bench --size 16777216 --chunks "" --single 16777216 > $O/single_16m.jsonl 2> $O/single_16m.err || fail single $?
            cat $O/single_16m.jsonl ;;
    phase) LZMA_AMD_LIB=$R/lzma-java_amd/build/prof/liblzma_mi355x.so timeout -k 10 300 python3 $R/tools/enc_scaling.py 16777216 1 > $O/phase_single_16m.txt 2>&1 || fail phase $?
           cat $O/phase_single_16m.txt ;;
  esac
done
