#!/bin/bash
# Profile passes over one bench step (bench.py --steps 1 --warmup 0: every
# kernel of the encode + decode path once, 1 GiB, 4096 streams).
#   1. phase profile of the parser (LZG_PROF build) at the same concurrency
#   2. kernel trace + stats
#   3. PMC passes (one counter group per run, never with other trace domains)
# Outputs are CSV; tools/pmc_reduce.py folds each pass into a small per-kernel
# table and the raw per-dispatch files are deleted (gpurun copies back <= 64 MiB).
# Any timeout / abort / crash ends the script.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-verify"
check() { echo "$1 rc=$2" >> $O/status.txt; case $2 in 0) ;; *) exit $2;; esac; }
reduce() { python3 $R/tools/pmc_reduce.py /tmp/prof_$1 > $O/$1.txt 2>&1; rm -rf /tmp/prof_$1; }
if [ "${SKIP_PHASE:-0}" = 0 ]; then
LZMA_AMD_LIB=$R/lzma-java_amd/build/prof/liblzma_mi355x.so timeout -k 10 200 python3 $R/tools/enc_scaling.py 262144 4096 > $O/phase.log 2>&1; check phase $?
fi
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_kt -o run -- python3 $B > $O/kt.log 2>&1; check kt $?; reduce kt
for pass in "A SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
            "B SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_IFETCH" \
            "F FETCH_SIZE" "W WRITE_SIZE" ${EXTRA_PASSES}; do
  set -- $pass; name=$1; shift
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d /tmp/prof_$name -o run -- python3 $B > $O/$name.log 2>&1; check $name $?; reduce $name
done
