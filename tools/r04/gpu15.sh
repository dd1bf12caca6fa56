#!/bin/bash
# round 4 GPU call 15: GPU parity subset (incl. the split-encode test) with the product, then the
# decoder's window flush as cached stores (build/exp_fl, LZG_DEC_FLUSH_NT=0) against the product
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04o
mkdir -p $O
cd $R
export TMPDIR=/tmp
F=$R/lzma-java_amd/build/exp_fl/liblzma_mi355x.so
P=$R/lzma-java_amd/build/liblzma_mi355x.so
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "not config4_shape and not full_1gib" > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for r in 1 2; do
  for L in $F $P; do
    LZMA_AMD_LIB=$L timeout -k 10 150 python3 tools/ab.py --reps 3 --parity 8 >> $O/ab.jsonl 2>> $O/ab.err || { echo "ab $L failed rc=$?"; tail -5 $O/ab.err; exit 1; }
    tail -1 $O/ab.jsonl | cut -c1-400
  done
done
for L in $F $P; do
  LZMA_AMD_LIB=$L timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-sample 0 --single-stream 0 --project-share 8 \
    > $O/s.json 2>> $O/share.err || { echo "share $L failed rc=$?"; tail -10 $O/share.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/s.json')); d['lib']='$L'; print(json.dumps(d))" >> $O/share8.jsonl
  python3 -c "import json; d=json.load(open('$O/s.json')); print('$L'[-40:], round(d['value'],1), round(d['ms_per_step'],1), d['verified'], {k: round(v['total_ms']/3,1) for k,v in d['kernels_ms'].items()})"
done
exit 0
