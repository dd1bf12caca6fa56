#!/bin/bash
# One PMC pass over a short encoder run (256 or 4096 streams): usage pmc_one.sh NAME NSTREAMS COUNTERS...
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
name=$1; ns=$2; shift 2
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d /tmp/prof_$name -o run -- python3 $R/tools/enc_scaling.py 262144 $ns > $O/$name.log 2>&1
rc=$?
python3 $R/tools/pmc_reduce.py /tmp/prof_$name > $O/$name.txt 2>&1
rm -rf /tmp/prof_$name
exit $rc
