#!/bin/bash
# Round 5: config 4's regime, one-off: ONE BENCH stream of ${MIB:-512} MiB at dict 2^26 L5
# encoded on the GPU and compared byte for byte with the oracle's Encoder.Code (on a host
# thread beside it): test_gpu_config4_shape_one_stream_longer_than_dict at that size. The
# 1 GiB stream of config 4 does not fit one gpurun call (1,200 s cap) at the measured rate.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05/config4
mkdir -p $O
cd $R
LZMA_CONFIG4_MIB=${MIB:-512} LZMA_CONFIG4_TIMEOUT=1100 timeout -k 10 1120 python -u -m pytest tests/test_gpu_parity.py -x -v -s \
  -k config4_shape --timeout-method thread > $O/config4_${MIB:-512}MiB.txt 2>&1 || { echo "config4 failed rc=$?"; tail -20 $O/config4_${MIB:-512}MiB.txt; exit 1; }
grep -E "config4 regime|passed|failed" $O/config4_${MIB:-512}MiB.txt
