#!/bin/bash
# round 4 GPU call 28: more scheduler / optimisation settings for the parse (build/flv2_*: -O2, no
# unclustered high-pressure reschedule, no clustered low-occupancy reschedule, metric bias 0)
# against the product: solo kernel times on BENCH (ab.py, 4 streams checked against the oracle per run)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04g
mkdir -p $O
cd $R
export TMPDIR=/tmp
B=$R/lzma-java_amd/build
for r in 1 2; do
  for L in $B/liblzma_mi355x.so $B/flv2_o2/liblzma_mi355x.so $B/flv2_nounc/liblzma_mi355x.so $B/flv2_noclu/liblzma_mi355x.so $B/flv2_bias0/liblzma_mi355x.so; do
    LZMA_AMD_LIB=$L timeout -k 10 150 python3 tools/ab.py --reps 3 --parity 4 >> $O/ab.jsonl 2>> $O/ab.err || { echo "ab $L failed rc=$?"; tail -5 $O/ab.err; exit 1; }
    python3 -c "import json; d=[json.loads(l) for l in open('$O/ab.jsonl')][-1]; k=d['kernels_ms']; print(d['lib'][-32:], round(d['MBps'],1), k.get('enc_parse'), k.get('mf_walk'), k.get('dec_stream'), d['parity'])"
  done
done
exit 0
