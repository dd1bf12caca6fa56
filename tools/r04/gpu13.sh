#!/bin/bash
# round 4 GPU call 13: the one-loop walk (a lane finishes a member and starts its next one
# within one tree step) -- GPU parity subset with build/exp_walk, then A/B against the product
# on BENCH and TEXT
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04m
mkdir -p $O
cd $R
export TMPDIR=/tmp
W=$R/lzma-java_amd/build/exp_walk/liblzma_mi355x.so
P=$R/lzma-java_amd/build/liblzma_mi355x.so
LZMA_AMD_LIB=$W timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "not config4_shape and not full_1gib" > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for r in 1 2; do
  for L in $W $P; do
    LZMA_AMD_LIB=$L timeout -k 10 150 python3 tools/ab.py --reps 3 --parity 8 >> $O/ab.jsonl 2>> $O/ab.err || { echo "ab $L failed rc=$?"; tail -5 $O/ab.err; exit 1; }
    tail -1 $O/ab.jsonl | cut -c1-400
  done
done
for L in $W $P; do
  LZMA_AMD_LIB=$L timeout -k 10 200 python3 tools/ab.py --data text --reps 2 --parity 4 >> $O/ab_text.jsonl 2>> $O/ab.err || { echo "ab text $L failed rc=$?"; tail -5 $O/ab.err; exit 1; }
  tail -1 $O/ab_text.jsonl | cut -c1-400
done
exit 0
