#!/bin/bash
# round 4 GPU call 19: PosInfo with a 4-positions-per-thread gather kernel (build/exp_pi) against the
# product: GPU parity subset, solo kernel times (ab.py) and the pipelined bench line, same box
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04s
mkdir -p $O
cd $R
export TMPDIR=/tmp
X=$R/lzma-java_amd/build/exp_pi/liblzma_mi355x.so
P=$R/lzma-java_amd/build/liblzma_mi355x.so
LZMA_AMD_LIB=$X timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "not config4_shape and not full_1gib" > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for L in $X $P; do
  LZMA_AMD_LIB=$L timeout -k 10 150 python3 tools/ab.py --reps 2 --parity 4 >> $O/ab.jsonl 2>> $O/ab.err || { echo "ab $L failed rc=$?"; tail -5 $O/ab.err; exit 1; }
  python3 -c "import json; d=[json.loads(l) for l in open('$O/ab.jsonl')][-1]; print(d['lib'][-30:], round(d['MBps'],1), {k: d['kernels_ms'][k] for k in d['kernels_ms'] if k.startswith('mf')}, d['parity'])"
done
for r in 1 2; do
  for L in $X $P; do
    LZMA_AMD_LIB=$L timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 --single-stream 0 > $O/b.json 2>> $O/bench.err || { echo "bench $L failed rc=$?"; tail -10 $O/bench.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b.json')); d['lib']='$L'; print(json.dumps(d))" >> $O/bench.jsonl
    python3 -c "import json; d=json.load(open('$O/b.json')); print('bench', '$L'[-30:], round(d['value'],1), round(d['ms_per_step'],1), d['verified'], {k: round(v['total_ms']/5,1) for k,v in d['kernels_ms'].items()})"
  done
done
exit 0
