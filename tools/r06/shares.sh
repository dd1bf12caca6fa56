#!/bin/bash
# Round 6 (from round 5) strong-scaling projection: rank 0's share of the 1 GiB bench buffer dealt over G GPUs,
# timed on one GPU with the default pipelined schedule (bench.py --project-share G; the parse
# fence is skipped at <= 8 streams per CU). One JSON line per G in gpurun_out/r06/shares.jsonl.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06
mkdir -p $O
for G in ${GS:-2 4 8}; do
  timeout -k 10 300 python3 $R/bench.py --project-share $G --pipeline ${PIPE:-split} --steps ${STEPS:-3} --warmup 1 --cpu-sample 0 --single-stream 0 --parity-streams 32 >> $O/${SH:-shares}.jsonl 2>> $O/${SH:-shares}.err || { echo "share $G failed rc=$?"; exit 1; }
  python3 -c "
import json; d = [json.loads(l) for l in open('$O/${SH:-shares}.jsonl')][-1]
print('G', d['projection_of_n_gpus'], 'value %.1f' % d['value'], 'ms %.1f' % d['ms_per_step'], 'verified', d['verified'], 'fence', d['parse_fence'], 'seq %.1f' % d['sequential']['value'], {k: round(v['total_ms'] / max(v['launches'], 1), 1) for k, v in d['kernels_ms'].items()})"
done
