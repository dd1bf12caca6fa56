#!/bin/bash
# One round-3 GPU call: A/B of the previous and current library (few-streams regime,
# then the bench batch), the -m gpu suite on the current library, then the probe.
#   usage: tools/r03_step.sh [ab] [tests] [probe]   (default: all)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03
mkdir -p $O
steps=${*:-ab tests probe}
for s in $steps; do
  case $s in
    ab) LIBS="lzma-java_amd/build/base/liblzma_mi355x.so lzma-java_amd/build/liblzma_mi355x.so" bash $R/tools/ab_r03.sh solo batch || exit 1 ;;
    tests) (cd $R && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1) || { echo "tests rc=$?"; tail -30 $O/gpu_tests.log; exit 1; }
           tail -3 $O/gpu_tests.log ;;
    probe) bash $R/tools/r03_probe.sh cpu strong || exit 1 ;;
  esac
done
