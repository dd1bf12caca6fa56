#!/bin/bash
# SQ counter passes over the batched decoder (tools/dec_scaling.py, 4096 x 256 KiB).
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
check() { echo "$1 rc=$2" >> $R/gpurun_out/pmc_dec_status.txt; case $2 in 124|134|137|139) exit $2;; esac; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $R/gpurun_out/pmcD1 -o run -- python3 $R/tools/dec_scaling.py 262144 4096 1 > $R/gpurun_out/pmcD1.log 2>&1; check D1 $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_VMEM -d $R/gpurun_out/pmcD2 -o run -- python3 $R/tools/dec_scaling.py 262144 4096 1 > $R/gpurun_out/pmcD2.log 2>&1; check D2 $?
