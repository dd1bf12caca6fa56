#!/bin/bash
# round 4 GPU call 2: concurrency probe after the mf_chains scan fix -> parity subset -> bench A/B sequential vs --overlap
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04b
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 240 python3 -u tools/concurrency_probe.py > $O/probe.json 2> $O/probe.err || { echo "probe failed rc=$?"; tail -8 $O/probe.err; exit 1; }
cat $O/probe.json
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "not config4_shape and not full_1gib" > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for r in 1 2; do
  for mode in "" "--overlap"; do
    timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --single-stream 0 --cpu-sample 0 --parity-streams 64 $mode \
      >> $O/bench_ab.jsonl 2>> $O/bench_ab.err || { echo "bench $mode failed rc=$?"; tail -20 $O/bench_ab.err; exit 1; }
    tail -1 $O/bench_ab.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$mode', d['value'], d['ms_per_step'], d['verified'], {k: round(v['total_ms']/5,1) for k,v in d['kernels_ms'].items()})"
  done
done
exit 0
