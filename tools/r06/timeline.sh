#!/bin/bash
# Round 6 (from round 5): kernel timeline of the pipelined bench (3 timed steps): rocprofv3 kernel trace,
# reduced by tools/timeline.py to the launches of the last steps, the GPU-idle gaps and the
# busy time per kernel. Output: gpurun_out/r06/${TAG:-tl}/timeline.txt
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06/${TAG:-tl}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/tl_kt -o run -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-sample 0 --single-stream 0 --no-verify ${BENCH_ARGS} > $O/bench.log 2>&1 || { echo "trace failed rc=$?"; tail -5 $O/bench.log; exit 1; }
python3 $R/tools/timeline.py /tmp/tl_kt --last ${LAST:-150} > $O/timeline.txt || exit 1
tail -40 $O/timeline.txt
