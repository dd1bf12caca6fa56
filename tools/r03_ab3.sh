#!/bin/bash
# three-way bench-batch A/B (base / batch-only experiment / current), twice, then the -m gpu suite
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03
mkdir -p $O
for i in 1 2; do
  LIBS="lzma-java_amd/build/base/liblzma_mi355x.so lzma-java_amd/build/nosolo/liblzma_mi355x.so lzma-java_amd/build/liblzma_mi355x.so" AB_ARGS="--parity 0" bash $R/tools/ab_r03.sh batch > /dev/null || exit 1
done
tail -6 $R/gpurun_out/ab/ab.jsonl
[ "$1" = tests ] || exit 0
(cd $R && timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1) || { echo "tests rc=$?"; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
