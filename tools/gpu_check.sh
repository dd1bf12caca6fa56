#!/bin/bash
# Standard GPU check: parity tests, then one bench line (no CPU baseline unless
# CPU=1). Each GPU step has its own time limit; the first failure ends the script.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
if [ "${TESTS:-1}" = 1 ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $O/gpu_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
fi
CS=0; [ "${CPU:-0}" = 1 ] && CS=33554432
timeout -k 10 400 python bench.py --cpu-sample $CS ${BENCH_ARGS} > $O/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value',d['value'],'enc',d['compress_MBps'],'dec',d['decompress_MBps'],'verified',d['verified']); print({k:round(v['total_ms']/d['steps'],1) for k,v in d['kernels_ms'].items()})"
