#!/bin/bash
# Round 6 A/B: bench.py with library variants, interleaved ROUNDS times. LIBS: space-separated
# library paths relative to the repo ("base" = the product build). Build the variants first,
# here on the CPU (they travel with the tree). One JSON line per run in gpurun_out/r06/$TAG.jsonl.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06
mkdir -p $O
cd $R
for r in $(seq ${ROUNDS:-2}); do
  for L in ${LIBS:-base}; do
    if [ "$L" = base ]; then LP=$R/lzma-java_amd/build/liblzma_mi355x.so; else LP=$R/$L; fi
    LZMA_AMD_LIB=$LP timeout -k 10 ${LIMIT:-240} python3 -u bench.py ${BENCH_ARGS:---steps 10 --warmup 2 --cpu-sample 0 --single-stream 0 --parity-streams 64} > $O/ab_one.json 2> $O/ab_one.err || { echo "bench $L failed rc=$?"; tail -5 $O/ab_one.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$O/ab_one.json')); d['lib'] = '$L'
open('$O/${TAG:-ab}.jsonl', 'a').write(json.dumps(d) + '\n')
print('$L', 'value %.1f ms %.1f verified %s' % (d['value'], d['ms_per_step'], d['verified']), {k: round(v['total_ms'] / max(v['launches'], 1), 1) for k, v in d['kernels_ms'].items()})"
  done
done
