#!/bin/bash
# Round-3 profiling steps (on the GPU box via gpurun); each GPU step has its own limit.
#   usage: tools/r03_prof.sh [pcs] [alloc] [abrep]
# pcs:   rocprofv3 PC sampling (stochastic, cycles) of the bench workload at 256 MiB
# alloc: lzma_encode/lzma_decode 100x on one context under --hip-trace --stats
# abrep: the bench batch A/B of base vs current library, 3 times each, interleaved
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
fail() { echo "$1 failed rc=$2"; exit $2; }
for s in ${*:-pcs alloc}; do
  case $s in
    pcs)
      timeout -k 10 60 rocprofv3 -L > $O/rocprof_list.txt 2>&1; grep -i -A12 "pc.sampl" $O/rocprof_list.txt | head -40
      timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
        --pc-sampling-interval 1048576 --output-format csv -d /tmp/pcs -o run -- \
        python3 $R/tools/ab.py --reps 1 --parity 0 --size 268435456 > $O/pcs.log 2>&1 || fail pcs $?
      find /tmp/pcs -name "*.csv" | head; mkdir -p $O/pcs && cp $(find /tmp/pcs -name "*.csv") $O/pcs/ ;;
    alloc)
      timeout -k 10 240 rocprofv3 --hip-trace --stats --output-format csv -d /tmp/alloc -o run -- \
        python3 $R/tools/c_abi_repeat.py 100 > $O/alloc.log 2>&1 || fail alloc $?
      mkdir -p $O/alloc && cp $(find /tmp/alloc -name "*stats*.csv") $O/alloc/ && cat $O/alloc/*hip_api_stats*.csv | head -30 ;;
    abrep)
      for i in 1 2 3; do
        LIBS="lzma-java_amd/build/base/liblzma_mi355x.so lzma-java_amd/build/liblzma_mi355x.so" AB_ARGS="--parity 0" bash $R/tools/ab_r03.sh batch > /dev/null || fail abrep $?
      done
      tail -6 $R/gpurun_out/ab/ab.jsonl ;;
  esac
done
