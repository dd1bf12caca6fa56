#!/bin/bash
# round 4 GPU call 27: the final product (per-source scheduler strategies) -- profiles (kernel stats, PMC traffic, issue), the full
# GPU suite, the default bench line (10 steps), config 3 (TEXT) and the strong-scaling shares
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04f
mkdir -p $O
cd $R
export TMPDIR=/tmp
PROF_OUT=$O bash tools/r04/prof.sh > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > $O/bench.json 2> $O/bench.err || { echo "bench failed rc=$?"; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', round(d['value'],1), round(d['ms_per_step'],1), d['verified'], d['single_stream']['parse_cycles_per_byte'])"
timeout -k 10 400 python -u bench.py --data text --steps 3 --warmup 1 --cpu-sample 0 --single-stream 0 > $O/bench_text.json 2> $O/bench_text.err || { echo "text bench failed rc=$?"; tail -10 $O/bench_text.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_text.json')); print('text', round(d['value'],1), round(d['ms_per_step'],1), d['verified'])"
for g in 2 4 8; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 --single-stream 0 --project-share $g \
    > $O/share_$g.json 2>> $O/share.err || { echo "share $g failed rc=$?"; tail -10 $O/share.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/share_$g.json')); print($g, round(d['value'],1), round(d['ms_per_step'],1), d['verified'])"
done
exit 0
