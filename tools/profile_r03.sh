#!/bin/bash
# Round-3 profile of the bench workload (run on the GPU box via gpurun).
#   usage: tools/profile_r03.sh [prof|sweep|text|all]
# prof:  kernel_stats.csv (rocprofv3 --kernel-trace --stats of one bench step),
#        traffic.json (separate FETCH_SIZE / WRITE_SIZE passes),
#        issue.json (SQ_INSTS_* issue counters, one pass)
# sweep: chunk sweep of the LzmaBench workload + one 64 MiB stream end to end
# text:  config 3 (TEXT, dict 2^28): bench line, chunk sweep, kernel stats and traffic
# Every GPU step has its own time limit; the first failure ends the script.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
what=${1:-all}
fail() { echo "$1 failed rc=$2"; exit $2; }
B="$R/bench.py --steps 1 --warmup 0 --cpu-sample 0 --single-stream 0 --no-verify"
WL='{"bytes_per_gpu": 1073741824, "chunk": 262144, "data": "bench", "dict_log": 26, "command": "bench.py --steps 1 --warmup 0 --cpu-sample 0 --single-stream 0 --no-verify"}'
if [ $what = prof -o $what = all ]; then
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_kt -o run -- python3 $B > $O/kt.log 2>&1 || fail kt $?
  python3 $R/tools/round_reduce.py stats /tmp/p_kt $O/kernel_stats.csv > /dev/null || fail reduce_kt $?
  rm -rf /tmp/p_kt
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d /tmp/p_f -o run -- python3 $B > $O/pmc_fetch.log 2>&1 || fail fetch $?
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d /tmp/p_w -o run -- python3 $B > $O/pmc_write.log 2>&1 || fail write $?
  python3 $R/tools/round_reduce.py traffic /tmp/p_f /tmp/p_w $O/traffic.json > /dev/null || fail reduce_traffic $?
  rm -rf /tmp/p_f /tmp/p_w
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_TEX_LOAD SQ_INSTS_TEX_STORE SQ_WAVES --output-format csv -d /tmp/p_i -o run -- python3 $B > $O/pmc_issue.log 2>&1 || fail issue $?
  python3 $R/tools/round_reduce.py counters /tmp/p_i $O/issue.json "$WL" > /dev/null || fail reduce_issue $?
  rm -rf /tmp/p_i
  echo prof done
fi
if [ $what = sweep -o $what = all ]; then
  timeout -k 10 600 python3 $R/tools/chunk_sweep.py --data bench > $O/sweep_bench.jsonl 2> $O/sweep_bench.err || fail sweep $?
  echo sweep done
fi
if [ $what = single ]; then
  timeout -k 10 600 python3 $R/tools/chunk_sweep.py --data bench --chunks "" --single 67108864 > $O/single_64m.jsonl 2> $O/single_64m.err || fail single $?
  echo single done
fi
if [ $what = phase ]; then
  make -s -C $R/lzma-java_amd prof > /dev/null || fail build_prof $?
  LZMA_AMD_LIB=$R/lzma-java_amd/build/prof/liblzma_mi355x.so timeout -k 10 200 python3 $R/tools/enc_scaling.py 262144 4096 > $O/phase.txt 2>&1 || fail phase $?
  echo phase done
fi
if [ $what = text -o $what = all ]; then
  timeout -k 10 400 python3 $R/bench.py --data text > $O/bench_text.log 2>&1 || fail bench_text $?
  BT="$R/bench.py --data text --steps 1 --warmup 0 --cpu-sample 0 --single-stream 0 --no-verify"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/t_kt -o run -- python3 $BT > $O/t_kt.log 2>&1 || fail t_kt $?
  python3 $R/tools/round_reduce.py stats /tmp/t_kt $O/text_kernel_stats.csv > /dev/null || fail reduce_t_kt $?
  rm -rf /tmp/t_kt
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d /tmp/t_f -o run -- python3 $BT > $O/t_fetch.log 2>&1 || fail t_fetch $?
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d /tmp/t_w -o run -- python3 $BT > $O/t_write.log 2>&1 || fail t_write $?
  python3 $R/tools/round_reduce.py traffic /tmp/t_f /tmp/t_w $O/text_traffic.json '{"bytes_per_gpu": 1073741824, "chunk": 262144, "data": "text", "dict_log": 28}' > /dev/null || fail reduce_t_traffic $?
  rm -rf /tmp/t_f /tmp/t_w
  timeout -k 10 400 python3 $R/tools/chunk_sweep.py --data text --chunks 262144,4194304 > $O/sweep_text.jsonl 2> $O/sweep_text.err || fail sweep_text $?
  echo text done
fi
