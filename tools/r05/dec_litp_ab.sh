#!/bin/bash
# Round 5: the decoder's plain literal trees in LDS at 16 streams per CU under the split
# schedule (experiment build, LZG_DEC_LITP_MAX=4096) against the product rule (<= 8 per CU),
# VARIANTS = build:litp_max pairs (build/exp_sr4: the sorts with 1024-item tiles),
# bench.py at N = 1, interleaved; one JSON line per run in gpurun_out/r05/declitp/ab.jsonl
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05/declitp
mkdir -p $O
for r in $(seq ${ROUNDS:-2}); do
  for V in ${VARIANTS:-exp:2048 exp:4096}; do
    B=${V%%:*}; M=${V##*:}
    LZMA_AMD_LIB=$R/lzma-java_amd/build/$B/liblzma_mi355x.so LZG_DEC_LITP_MAX=$M timeout -k 10 300 python3 $R/bench.py --steps 6 --warmup 1 --cpu-sample 0 --single-stream 0 --parity-streams 32 >> $O/ab.jsonl 2>> $O/ab.err || { echo "bench $M failed rc=$?"; exit 1; }
    python3 -c "
import json; d = [json.loads(l) for l in open('$O/ab.jsonl')][-1]
print('$B litp_max $M', 'value %.1f' % d['value'], 'ms %.1f' % d['ms_per_step'], 'verified', d['verified'], {k: round(v['total_ms'] / max(v['launches'], 1), 1) for k, v in d['kernels_ms'].items()})"
  done
done
