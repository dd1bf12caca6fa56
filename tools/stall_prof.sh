#!/bin/bash
# Stall/issue counters of the bench workload's kernels (on the GPU box via gpurun):
# where a latency-bound wave spends its cycles. One --pmc pass per counter set.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/stall
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-verify"
WL='{"bytes_per_gpu": 1073741824, "chunk": 262144, "data": "bench", "dict_log": 26, "command": "bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-verify"}'
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || echo "list rc=$?"
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $set --output-format csv -d /tmp/s_$i -o run -- python3 $B > $O/pass_$i.log 2>&1 || { echo "pass $i ($set) rc=$?"; tail -5 $O/pass_$i.log; exit 1; }
  python3 $R/tools/round_reduce.py counters /tmp/s_$i $O/stall_$i.json "$WL" > /dev/null || { echo "reduce $i failed"; exit 1; }
  rm -rf /tmp/s_$i
  echo "pass $i done"
done
