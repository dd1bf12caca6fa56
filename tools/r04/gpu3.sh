#!/bin/bash
# round 4 GPU call 3: the two-wave parser (build/exp1) -- parity subset, one-wave vs two-wave on few
# streams per CU and one long stream, and the 4096-stream batch A/B against the current product
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04c
mkdir -p $O
cd $R
export TMPDIR=/tmp
EXP=$R/lzma-java_amd/build/exp1/liblzma_mi355x.so
LZMA_AMD_LIB=$EXP timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "not config4_shape and not full_1gib" > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for w in 0 1; do
  LZMA_AMD_LIB=$EXP LZG_ENC_W2=$w timeout -k 10 240 python3 tools/r04/w2_probe.py 4194304 1 1 >> $O/w2.jsonl 2>> $O/w2.err || { echo "w2 single $w failed rc=$?"; tail -5 $O/w2.err; exit 1; }
  tail -1 $O/w2.jsonl
done
for w in 0 1; do
  LZMA_AMD_LIB=$EXP LZG_ENC_W2=$w timeout -k 10 240 python3 tools/r04/w2_probe.py 262144 256,512,1024,2048 8 >> $O/w2.jsonl 2>> $O/w2.err || { echo "w2 batch $w failed rc=$?"; tail -5 $O/w2.err; exit 1; }
  tail -4 $O/w2.jsonl
done
for r in 1 2; do
  for L in lzma-java_amd/build/liblzma_mi355x.so lzma-java_amd/build/exp1/liblzma_mi355x.so; do
    LZMA_AMD_LIB=$R/$L timeout -k 10 150 python3 tools/ab.py --reps 3 --parity 8 >> $O/ab.jsonl 2>> $O/ab.err || { echo "ab $L failed rc=$?"; tail -5 $O/ab.err; exit 1; }
    tail -1 $O/ab.jsonl | cut -c1-330
  done
done
exit 0
