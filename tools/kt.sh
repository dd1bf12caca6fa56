#!/bin/bash
# rocprofv3 kernel trace + stats of one bench step (on the GPU box via gpurun); out: gpurun_out/kt/kernel_stats.csv
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/kt
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt -o run -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-verify ${KT_ARGS:-} > $O/kt.log 2>&1 || { echo "kt failed rc=$?"; tail -5 $O/kt.log; exit 1; }
python3 $R/tools/round_reduce.py stats /tmp/kt $O/kernel_stats.csv > /dev/null || exit 1
cat $O/kernel_stats.csv
