#!/bin/bash
# Round-4 profile of the bench workload (GPU box, via gpurun): writes gpurun_out/r04/
#   kernel_stats.csv  rocprofv3 --kernel-trace --stats of one bench step
#   traffic.json      separate FETCH_SIZE / WRITE_SIZE passes (per launch)
#   issue.json        SQ_INSTS_* issue counters (one pass)
# Every GPU step has its own time limit; the first failure ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=${PROF_OUT:-$R/gpurun_out/r04}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
fail() { echo "$1 failed rc=$2"; exit $2; }
B="$R/bench.py --steps 1 --warmup 0 --cpu-sample 0 --single-stream 0 --no-verify"
WL='{"bytes_per_gpu": 1073741824, "chunk": 262144, "data": "bench", "dict_log": 26, "command": "bench.py --steps 1 --warmup 0 --cpu-sample 0 --single-stream 0 --no-verify"}'
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_kt -o run -- python3 $B > $O/kt.log 2>&1 || fail kt $?
python3 $R/tools/round_reduce.py stats /tmp/p_kt $O/kernel_stats.csv > /dev/null || fail reduce_kt $?
rm -rf /tmp/p_kt
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d /tmp/p_f -o run -- python3 $B > $O/pmc_fetch.log 2>&1 || fail fetch $?
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d /tmp/p_w -o run -- python3 $B > $O/pmc_write.log 2>&1 || fail write $?
python3 $R/tools/round_reduce.py traffic /tmp/p_f /tmp/p_w $O/traffic.json "$WL" > /dev/null || fail reduce_traffic $?
rm -rf /tmp/p_f /tmp/p_w
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_TEX_LOAD SQ_INSTS_TEX_STORE SQ_WAVES --output-format csv -d /tmp/p_i -o run -- python3 $B > $O/pmc_issue.log 2>&1 || fail issue $?
python3 $R/tools/round_reduce.py counters /tmp/p_i $O/issue.json "$WL" > /dev/null || fail reduce_issue $?
rm -rf /tmp/p_i
echo prof done
head -12 $O/kernel_stats.csv
