#!/bin/bash
# round 4 GPU call 5: build/exp3 (nx fs prefetch, no LDS gather window) vs the product
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04e
mkdir -p $O
cd $R
export TMPDIR=/tmp
E3=$R/lzma-java_amd/build/exp3/liblzma_mi355x.so
P=$R/lzma-java_amd/build/liblzma_mi355x.so
LZMA_AMD_LIB=$E3 timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "not config4_shape and not full_1gib" > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for L in $P $E3; do
  LZMA_AMD_LIB=$L timeout -k 10 240 python3 tools/r04/w2_probe.py 4194304 1 1 > $O/p.json 2>> $O/w.err || { echo "probe failed"; tail -5 $O/w.err; exit 1; }
  sed "s|^{|{\"lib\": \"$L\", |" $O/p.json >> $O/w.jsonl; tail -1 $O/w.jsonl | cut -c1-260
done
for r in 1 2; do
  for L in $P $E3; do
    LZMA_AMD_LIB=$L timeout -k 10 150 python3 tools/ab.py --reps 3 --parity 8 >> $O/ab.jsonl 2>> $O/ab.err || { echo "ab $L failed rc=$?"; tail -5 $O/ab.err; exit 1; }
    tail -1 $O/ab.jsonl | cut -c1-330
  done
done
exit 0
