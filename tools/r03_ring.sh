#!/bin/bash
# Round-3 _optimum ring: A/B (HEAD library vs ring library, BENCH and TEXT, 8 streams
# checked against the oracle each), the TEXT/BENCH phase profile, then the GPU tests.
#   usage: tools/r03_ring.sh [ab] [phase] [tests]
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
fail() { echo "$1 failed rc=$2"; exit $2; }
for s in ${*:-ab phase tests}; do
  case $s in
    ab)
      for d in text bench; do
        LIBS="${AB_LIBS:-lzma-java_amd/build/head/liblzma_mi355x.so lzma-java_amd/build/liblzma_mi355x.so}" \
          AB_ARGS="--data $d --reps 2 --parity 8" bash $R/tools/ab_r03.sh batch > /dev/null || fail ab_$d $?
      done
      cat $R/gpurun_out/ab/ab.jsonl ;;
    phase)
      bash $R/tools/r03_text.sh phase > /dev/null || fail phase $?
      grep -E "get_optimum|relax|state|n_spill|n_pos|enc_parse" $O/phase_text.txt $O/phase_bench.txt ;;
    tests)
      cd $R && timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 700 --timeout-method thread \
        > $O/gpu_tests_ring.log 2>&1 || { tail -30 $O/gpu_tests_ring.log; fail tests $?; }
      tail -5 $O/gpu_tests_ring.log ;;
  esac
done
