#!/bin/bash
# round 4 GPU call 8: per-phase cycle profile of the parse (LZG_PROF build): one 4 MiB stream, 256 and 4096 streams of 256 KiB
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04h
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
fail() { echo "$1 failed rc=$2"; exit $2; }
L=$R/lzma-java_amd/build/prof/liblzma_mi355x.so
LZMA_AMD_LIB=$L timeout -k 10 200 python3 $R/tools/enc_scaling.py 4194304 1 bench > $O/phase_single.txt 2>&1 || fail single $?
LZMA_AMD_LIB=$L timeout -k 10 200 python3 $R/tools/enc_scaling.py 262144 256,4096 bench > $O/phase_batch.txt 2>&1 || fail batch $?
tail -n 24 $O/phase_single.txt; tail -n 48 $O/phase_batch.txt
