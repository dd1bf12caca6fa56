#!/bin/bash
# round 4 GPU call 17: the walk's register diet (32-bit indices, no per-lane stream pointers:
# 121 -> 104 VGPRs; build/exp_diet) and the same with 5 waves per SIMD (build/exp_diet5,
# LZG_WALK_WAVES=5: 96 VGPRs, 12 B scratch) against the product, BENCH and TEXT; parity subset
# with exp_diet5 first
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04q
mkdir -p $O
cd $R
export TMPDIR=/tmp
D=$R/lzma-java_amd/build/exp_diet/liblzma_mi355x.so
D5=$R/lzma-java_amd/build/exp_diet5/liblzma_mi355x.so
P=$R/lzma-java_amd/build/liblzma_mi355x.so
LZMA_AMD_LIB=$D5 timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "not config4_shape and not full_1gib" > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for r in 1 2; do
  for L in $D5 $D $P; do
    LZMA_AMD_LIB=$L timeout -k 10 150 python3 tools/ab.py --reps 2 --parity 4 >> $O/ab.jsonl 2>> $O/ab.err || { echo "ab $L failed rc=$?"; tail -5 $O/ab.err; exit 1; }
    python3 -c "import json; d=[json.loads(l) for l in open('$O/ab.jsonl')][-1]; print(d['lib'][-30:], round(d['MBps'],1), d['kernels_ms']['mf_walk'], d['parity'])"
  done
done
for L in $D5 $D $P; do
  LZMA_AMD_LIB=$L timeout -k 10 200 python3 tools/ab.py --data text --reps 2 --parity 4 >> $O/ab_text.jsonl 2>> $O/ab.err || { echo "ab text $L failed rc=$?"; tail -5 $O/ab.err; exit 1; }
  python3 -c "import json; d=[json.loads(l) for l in open('$O/ab_text.jsonl')][-1]; print('text', d['lib'][-30:], round(d['MBps'],1), d['kernels_ms']['mf_walk'], d['parity'])"
done
# the product (decoder literal trees in LDS only up to 8 streams per CU): the pipelined bench line
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 --single-stream 0 > $O/bench.json 2> $O/bench.err || { echo "bench failed rc=$?"; tail -10 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', round(d['value'],1), round(d['ms_per_step'],1), d['verified'], {k: round(v['total_ms']/5,1) for k,v in d['kernels_ms'].items()})"
exit 0
