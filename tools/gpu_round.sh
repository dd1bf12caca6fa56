#!/bin/bash
# One GPU call: the -m gpu suite, the default bench line, then the kernel/PMC profile.
#   usage: tools/gpu_round.sh [tests] [bench] [prof]   (default: all three)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02
mkdir -p $O
steps=${*:-tests bench prof}
for s in $steps; do
  case $s in
    tests) (cd $R && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1) || { echo "tests rc=$?"; tail -30 $O/gpu_tests.log; exit 1; }
           tail -3 $O/gpu_tests.log ;;
    bench) (cd $R && timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err) || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 1; }
           cat $O/bench.json ;;
    prof)  bash $R/tools/profile_r02.sh prof || exit 1 ;;
  esac
done
