#!/bin/bash
# A/B of library builds on the bench workload, interleaved: tools/ab_libs.sh "libA libB ..." [rounds] [ab.py args]
# one JSON line per run (tools/ab.py) appended to gpurun_out/ab/ab_libs.jsonl; each run has its own time limit
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/ab
ROUNDS=${2:-2}
for r in $(seq $ROUNDS); do
  for L in $1; do
    LZMA_AMD_LIB=$R/$L timeout -k 10 120 python3 $R/tools/ab.py ${3:---reps 2 --parity 8} >> $R/gpurun_out/ab/ab_libs.jsonl 2>> $R/gpurun_out/ab/ab_libs.err || { echo "ab $L failed rc=$?"; exit 1; }
    tail -1 $R/gpurun_out/ab/ab_libs.jsonl | cut -c1-300
  done
done
