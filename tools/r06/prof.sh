#!/bin/bash
# Round 6 profile of one bench step (GPU box, via gpurun), DATA=bench (default) or text:
#   ${P}kernel_stats.csv  rocprofv3 --kernel-trace --stats of one bench step
#   ${P}traffic.json      separate FETCH_SIZE / WRITE_SIZE passes (per launch)
#   ${P}issue.json        SQ_INSTS_* issue counters (one pass)
# with P = "" (bench) or "text_" under gpurun_out/r06/prof/. Every GPU step has its own time
# limit; the first failure ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
DATA=${DATA:-bench}
O=$R/gpurun_out/r06/prof
mkdir -p $O
P=""; DL=26; [ "$DATA" = text ] && { P="text_"; DL=28; }
cd /tmp && export TMPDIR=/tmp
fail() { echo "$1 failed rc=$2"; exit $2; }
B="$R/bench.py --data $DATA --steps 1 --warmup 0 --cpu-sample 0 --single-stream 0 --no-verify"
WL="{\"bytes_per_gpu\": 1073741824, \"chunk\": 262144, \"data\": \"$DATA\", \"dict_log\": $DL, \"command\": \"bench.py --data $DATA --steps 1 --warmup 0 --cpu-sample 0 --single-stream 0 --no-verify\"}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_kt -o run -- python3 $B > $O/${P}kt.log 2>&1 || fail kt $?
python3 $R/tools/round_reduce.py stats /tmp/p_kt $O/${P}kernel_stats.csv > /dev/null || fail reduce_kt $?
rm -rf /tmp/p_kt
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d /tmp/p_f -o run -- python3 $B > $O/${P}pmc_fetch.log 2>&1 || fail fetch $?
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d /tmp/p_w -o run -- python3 $B > $O/${P}pmc_write.log 2>&1 || fail write $?
python3 $R/tools/round_reduce.py traffic /tmp/p_f /tmp/p_w $O/${P}traffic.json "$WL" > /dev/null || fail reduce_traffic $?
rm -rf /tmp/p_f /tmp/p_w
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_TEX_LOAD SQ_INSTS_TEX_STORE SQ_WAVES --output-format csv -d /tmp/p_i -o run -- python3 $B > $O/${P}pmc_issue.log 2>&1 || fail issue $?
python3 $R/tools/round_reduce.py counters /tmp/p_i $O/${P}issue.json "$WL" > /dev/null || fail reduce_issue $?
rm -rf /tmp/p_i
echo "prof $DATA done"
head -12 $O/${P}kernel_stats.csv
