#!/bin/bash
# round 4 GPU call 4: literal coders in LDS for few-stream launches (build/exp2) vs build/exp1
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04d
mkdir -p $O
cd $R
export TMPDIR=/tmp
E1=$R/lzma-java_amd/build/exp1/liblzma_mi355x.so
E2=$R/lzma-java_amd/build/exp2/liblzma_mi355x.so
LZMA_AMD_LIB=$E2 timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "not config4_shape and not full_1gib" > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
run() {  # lib label env...
  local L=$1; shift; local tag=$1; shift
  env "$@" LZMA_AMD_LIB=$L timeout -k 10 240 python3 tools/r04/w2_probe.py 4194304 1 1 > $O/p.json 2>> $O/w.err || { echo "probe $tag failed"; tail -5 $O/w.err; exit 1; }
  sed "s/^{/{\"tag\": \"$tag\", /" $O/p.json >> $O/w.jsonl; tail -1 $O/w.jsonl | cut -c1-220
}
run $E1 exp1_w1 LZG_ENC_W2=0
run $E2 exp2_w1 LZG_ENC_W2=0
run $E2 exp2_w2 LZG_ENC_W2=1
for L in $E1 $E2; do
  LZMA_AMD_LIB=$L timeout -k 10 240 python3 tools/r04/w2_probe.py 262144 256,512,1024 4 > $O/p.json 2>> $O/w.err || { echo "batch failed"; exit 1; }
  sed "s|^{|{\"lib\": \"$(basename $(dirname $L))\", |" $O/p.json >> $O/w.jsonl; tail -3 $O/w.jsonl | cut -c1-220
done
exit 0
