#!/bin/bash
# Kernel stats and per-kernel HBM traffic of one bench step (run on the GPU box
# via gpurun): kernel_stats.csv, traffic.json under gpurun_out/$1 (default traffic).
# Every GPU step has its own time limit; the first failure ends the script.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-traffic}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-verify ${BENCH_ARGS}"
fail() { echo "$1 failed rc=$2"; exit $2; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_kt -o run -- python3 $B > $O/kt.log 2>&1 || fail kt $?
python3 $R/tools/round_reduce.py stats /tmp/prof_kt $O/kernel_stats.csv || fail reduce_kt $?
rm -rf /tmp/prof_kt
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d /tmp/prof_f -o run -- python3 $B > $O/pmc_fetch.log 2>&1 || fail fetch $?
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d /tmp/prof_w -o run -- python3 $B > $O/pmc_write.log 2>&1 || fail write $?
python3 $R/tools/round_reduce.py traffic /tmp/prof_f /tmp/prof_w $O/traffic.json || fail reduce_traffic $?
rm -rf /tmp/prof_f /tmp/prof_w
echo traffic done
