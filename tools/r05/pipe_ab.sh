#!/bin/bash
# Round 5: bench step under the two pipelined schedules (decode beside the next match finder;
# split: also the range coder beside it), interleaved ROUNDS times; one JSON line per run in
# gpurun_out/r05/${TAG:-pipe}/pipe.jsonl
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05/${TAG:-pipe}
mkdir -p $O
for r in $(seq ${ROUNDS:-2}); do
  for P in decode split; do
    timeout -k 10 300 python3 $R/bench.py --pipeline $P --steps ${STEPS:-4} --warmup 1 --cpu-sample 0 --single-stream 0 --parity-streams 32 $BENCH_ARGS >> $O/pipe.jsonl 2>> $O/pipe.err || { echo "bench $P failed rc=$?"; exit 1; }
    python3 -c "
import json; d = [json.loads(l) for l in open('$O/pipe.jsonl')][-1]
print('$P', 'value %.1f' % d['value'], 'ms %.1f' % d['ms_per_step'], 'verified', d['verified'])"
  done
done
