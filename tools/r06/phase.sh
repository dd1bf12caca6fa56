#!/bin/bash
# Build first, here on the CPU: make -C lzma-java_amd prof (build/prof/liblzma_mi355x.so travels with the tree).
# Round 6 (from round 5): per-phase cycle profile of the parse (LZG_PROF build, `make -C lzma-java_amd prof`):
# one 4 MiB stream, then 256 and 4096 streams of 256 KiB (BENCH data, dict 2^26, L5)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06/${TAG:-phase}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
fail() { echo "$1 failed rc=$2"; exit $2; }
L=${LIB:-$R/lzma-java_amd/build/prof/liblzma_mi355x.so}
LZMA_AMD_LIB=$L timeout -k 10 200 python3 $R/tools/enc_scaling.py 4194304 1 bench > $O/phase_single.txt 2>&1 || fail single $?
LZMA_AMD_LIB=$L timeout -k 10 200 python3 $R/tools/enc_scaling.py 262144 256,4096 bench > $O/phase_batch.txt 2>&1 || fail batch $?
cat $O/phase_single.txt; cat $O/phase_batch.txt
