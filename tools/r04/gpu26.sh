#!/bin/bash
# round 4 GPU call 26: per-source scheduler strategies (mf iterative-ilp, dec max-ilp; build/exp_fl)
# against the product: GPU parity subset, solo kernel times on BENCH and TEXT
# (ab.py), the pipelined bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04z
mkdir -p $O
cd $R
export TMPDIR=/tmp
X=$R/lzma-java_amd/build/exp_fl/liblzma_mi355x.so
P=$R/lzma-java_amd/build/liblzma_mi355x.so
LZMA_AMD_LIB=$X timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "not config4_shape and not full_1gib" > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for r in 1 2; do
  for L in $X $P; do
    LZMA_AMD_LIB=$L timeout -k 10 150 python3 tools/ab.py --reps 3 --parity 4 >> $O/ab.jsonl 2>> $O/ab.err || { echo "ab $L failed rc=$?"; tail -5 $O/ab.err; exit 1; }
    python3 -c "import json; d=[json.loads(l) for l in open('$O/ab.jsonl')][-1]; print(d['lib'][-30:], round(d['MBps'],1), d['kernels_ms'].get('mf_walk'), d['kernels_ms'].get('mf_sort'), d['parity'])"
  done
done
for L in $X $P; do
  LZMA_AMD_LIB=$L timeout -k 10 200 python3 tools/ab.py --data text --reps 2 --parity 2 >> $O/ab_text.jsonl 2>> $O/ab.err || { echo "ab text $L failed rc=$?"; tail -5 $O/ab.err; exit 1; }
  python3 -c "import json; d=[json.loads(l) for l in open('$O/ab_text.jsonl')][-1]; print('text', d['lib'][-30:], round(d['MBps'],1), d['kernels_ms'].get('mf_walk'), d['kernels_ms'].get('mf_sort'), d['parity'])"
done
for L in $X $P; do
  LZMA_AMD_LIB=$L timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 --single-stream 0 > $O/b.json 2>> $O/bench.err || { echo "bench $L failed rc=$?"; tail -10 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b.json')); d['lib']='$L'; print(json.dumps(d))" >> $O/bench.jsonl
  python3 -c "import json; d=json.load(open('$O/b.json')); print('bench', '$L'[-30:], round(d['value'],1), round(d['ms_per_step'],1), d['verified'])"
done
exit 0
