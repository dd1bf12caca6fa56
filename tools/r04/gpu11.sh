#!/bin/bash
# round 4 GPU call 11: the split encode (range coder on its own stream beside the next batch's
# match finder) -- GPU parity subset, then bench.py A/B: split vs decode-only overlap vs sequential
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04k
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "not config4_shape and not full_1gib" > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for r in 1 2; do
  for mode in split decode; do
    timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 --single-stream 0 --pipeline $mode \
      > $O/b.json 2>> $O/bench.err || { echo "bench $mode failed rc=$?"; tail -20 $O/bench.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b.json')); d['pipeline']='$mode'; print(json.dumps(d))" >> $O/ab.jsonl
    python3 -c "import json; d=json.load(open('$O/b.json')); print('$mode', round(d['value'],1), round(d['ms_per_step'],1), d['verified'], {k: round(v['total_ms']/5,1) for k,v in d['kernels_ms'].items()})"
  done
done
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 --single-stream 0 --sequential > $O/b.json 2>> $O/bench.err || { echo "bench seq failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b.json')); d['pipeline']='sequential'; print(json.dumps(d))" >> $O/ab.jsonl
python3 -c "import json; d=json.load(open('$O/b.json')); print('sequential', round(d['value'],1), round(d['ms_per_step'],1), d['verified'])"
exit 0
