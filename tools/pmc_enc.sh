#!/bin/bash
# PMC passes over the encoder workload (tools/enc_scaling.py, 256 x 256 KiB).
# Counter passes run separately (never combined with other trace domains).
# A pass that fails for a bad counter name is recorded and the next pass
# runs; a timeout, abort or crash ends the script.
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
check() { echo "$1 rc=$2" >> $R/gpurun_out/pmc_status.txt; case $2 in 124|134|137|139) exit $2;; esac; }
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1; check list $?
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $R/gpurun_out/pmcA -o run -- python3 $R/tools/enc_scaling.py 262144 256 > $R/gpurun_out/pmcA.log 2>&1; check A $?
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_IFETCH -d $R/gpurun_out/pmcB -o run -- python3 $R/tools/enc_scaling.py 262144 256 > $R/gpurun_out/pmcB.log 2>&1; check B $?
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES -d $R/gpurun_out/pmcC -o run -- python3 $R/tools/enc_scaling.py 262144 256 > $R/gpurun_out/pmcC.log 2>&1; check C $?
