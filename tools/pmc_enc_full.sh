#!/bin/bash
# One SQ counter pass over the encoder at full occupancy (4096 x 256 KiB).
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $R/gpurun_out/pmcF -o run -- python3 $R/tools/enc_scaling.py 262144 4096 > $R/gpurun_out/pmcF.log 2>&1
