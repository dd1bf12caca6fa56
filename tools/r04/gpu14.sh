#!/bin/bash
# round 4 GPU call 14: fresh profiles of the product (kernel stats, PMC traffic, issue), then
# VERDICT r03's config-4 check: one 256 MiB BENCH stream at dict 2^26 L5, byte-equal to the oracle
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04n
mkdir -p $O
cd $R
export TMPDIR=/tmp
PROF_OUT=$O bash tools/r04/prof.sh > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
tail -12 $O/prof.log
cd $R
LZMA_CONFIG4_MIB=256 timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -s -v --timeout 980 \
  --timeout-method thread -k config4_shape > $O/config4_256.txt 2>&1 || { echo "config4 failed rc=$?"; tail -30 $O/config4_256.txt; exit 1; }
grep -E "config4 regime|passed|failed" $O/config4_256.txt
exit 0
