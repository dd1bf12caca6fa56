#!/bin/bash
# round 4 GPU call 9: the single-wave pipelined parse (enc.hip SP) -- parity, then SP off / on
# at one stream and few streams per CU, and the 4096-stream batch against the round's
# previous build (build/exp2: the plain kernel before the gather split)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04i
mkdir -p $O
cd $R
export TMPDIR=/tmp
E2=$R/lzma-java_amd/build/exp2/liblzma_mi355x.so
P=$R/lzma-java_amd/build/liblzma_mi355x.so
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "not config4_shape and not full_1gib" > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for sp in 0 1; do
  LZG_ENC_SP=$sp timeout -k 10 240 python3 tools/r04/w2_probe.py 4194304 1 1 >> $O/sp.jsonl 2>> $O/sp.err || { echo "probe failed"; tail -5 $O/sp.err; exit 1; }
  tail -1 $O/sp.jsonl | cut -c1-260
done
for sp in 0 1; do
  LZG_ENC_SP=$sp timeout -k 10 240 python3 tools/r04/w2_probe.py 262144 256,512,1024 8 >> $O/sp.jsonl 2>> $O/sp.err || { echo "probe failed"; tail -5 $O/sp.err; exit 1; }
  tail -3 $O/sp.jsonl | cut -c1-200
done
for r in 1 2; do
  for L in $P $E2; do
    LZMA_AMD_LIB=$L timeout -k 10 150 python3 tools/ab.py --reps 3 --parity 8 >> $O/ab.jsonl 2>> $O/ab.err || { echo "ab $L failed rc=$?"; tail -5 $O/ab.err; exit 1; }
    tail -1 $O/ab.jsonl | cut -c1-330
  done
done
exit 0
