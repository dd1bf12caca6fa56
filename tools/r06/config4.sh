#!/bin/bash
# Round 6: one call of config 4's sliced run (tools/r06/config4_sliced.py). STATE_IN: the
# checkpoint directory the previous call left (committed under profiles/r06/config4_state/);
# the new one goes to gpurun_out/r06/config4/$TAG. With TEST=1 the GPU session test runs first.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06/config4/${TAG:-c0}
mkdir -p $O
cd $R
if [ -n "$TEST" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -k session --timeout 280 --timeout-method thread > $O/session_test.txt 2>&1 || { echo "session test failed rc=$?"; tail -30 $O/session_test.txt; exit 1; }
  grep -E "passed|failed" $O/session_test.txt
fi
timeout -k 10 ${LIMIT:-1000} python -u tools/r06/config4_sliced.py --budget ${BUDGET:-900} ${STATE_IN:+--state-in $STATE_IN} --state-out $O > $O/run.log 2>&1 || { echo "config4 call failed rc=$?"; tail -20 $O/run.log; exit 1; }
tail -4 $O/run.log
