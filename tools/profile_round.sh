#!/bin/bash
# Round profile of the bench workload (run on the GPU box via gpurun):
#   bench.json          the default bench line (with the CPU baseline)
#   kernel_stats.csv    rocprofv3 --kernel-trace --stats of one bench step
#   traffic.json        per-kernel HBM bytes per launch from separate FETCH_SIZE / WRITE_SIZE passes
#   scaling.txt         parser and decoder time at 1, 4 and 16 streams per CU
# Every GPU step has its own time limit; the first failure ends the script.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/round
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-verify"
fail() { echo "$1 failed rc=$2"; exit $2; }
timeout -k 10 500 python3 $R/bench.py > $O/bench.log 2>&1 || fail bench $?
grep '^{' $O/bench.log > $O/bench.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_kt -o run -- python3 $B > $O/kt.log 2>&1 || fail kt $?
python3 $R/tools/round_reduce.py stats /tmp/prof_kt $O/kernel_stats.csv || fail reduce_kt $?
rm -rf /tmp/prof_kt
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d /tmp/prof_f -o run -- python3 $B > $O/pmc_fetch.log 2>&1 || fail fetch $?
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d /tmp/prof_w -o run -- python3 $B > $O/pmc_write.log 2>&1 || fail write $?
python3 $R/tools/round_reduce.py traffic /tmp/prof_f /tmp/prof_w $O/traffic.json || fail reduce_traffic $?
rm -rf /tmp/prof_f /tmp/prof_w
cd $R
for n in 256 1024 4096; do
  timeout -k 10 200 python3 tools/enc_scaling.py 262144 $n 2>&1 | grep streams >> $O/scaling.txt || fail enc_scaling $?
  timeout -k 10 200 python3 tools/dec_scaling.py 262144 $n 1 2>&1 | grep streams >> $O/scaling.txt || fail dec_scaling $?
done
echo profile done
