#!/bin/bash
# round 4 GPU call 7: profiles of the product (kernel stats, traffic, issue), config 3 (TEXT) bench line,
# strong-scaling share projections (rank 0's share of G = 2, 4, 8 on this one GPU, pipelined schedule)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04g
mkdir -p $O
cd $R
export TMPDIR=/tmp
bash tools/r04/prof.sh || { echo "prof failed"; exit 1; }
for g in 2 4 8; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 --single-stream 0 --project-share $g \
    > $O/share_$g.json 2>> $O/share.err || { echo "share $g failed rc=$?"; tail -10 $O/share.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/share_$g.json')); print($g, round(d['value'],1), round(d['ms_per_step'],1), d['verified'], {k: round(v['total_ms']/5,1) for k,v in d['kernels_ms'].items()})"
done
timeout -k 10 400 python -u bench.py --data text --steps 3 --warmup 1 --cpu-sample 0 --single-stream 0 \
  > $O/bench_text.json 2> $O/bench_text.err || { echo "text bench failed rc=$?"; tail -10 $O/bench_text.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_text.json')); print('text', round(d['value'],1), round(d['ms_per_step'],1), d['verified'], {k: round(v['total_ms']/3,1) for k,v in d['kernels_ms'].items()})"
exit 0
