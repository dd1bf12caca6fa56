#!/bin/bash
# Round 6: the driver's GPU tier by hand: the -m gpu suite, then the driver's bench command
# (20 steps, 5 warm-up). Outputs under gpurun_out/r06/$TAG/; each GPU step has its own limit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06/${TAG:-full}
mkdir -p $O
cd $R
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 ${TEST_LIMIT:-800} python -u -m pytest tests -m gpu -x -v --timeout 700 --timeout-method thread ${PYTEST_ARGS} > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gpu_tests.txt; exit 1; }
  tail -3 $O/gpu_tests.txt
fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 ${BENCH_LIMIT:-500} python -u bench.py ${BENCH_ARGS:---gpus 1 --steps 20 --warmup 5} > $O/bench.json 2> $O/bench.err || { echo "bench failed rc=$?"; tail -20 $O/bench.err; exit 1; }
  python3 -c "
import json; d = json.load(open('$O/bench.json'))
print('value %.1f MB/s, %.1f ms/step, verified %s' % (d['value'], d['ms_per_step'], d['verified']))
print('sequential', json.dumps(d['sequential']))
print('kernels', {k: round(v['total_ms'] / max(v['launches'], 1), 1) for k, v in d['kernels_ms'].items()})
s = d.get('single_stream') or {}
print('single', {k: s.get(k) for k in ('parse_cycles_per_byte', 'gpu_compress_MBps', 'equals_oracle', 'roundtrip_ok')})
"
fi
