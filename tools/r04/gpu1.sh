#!/bin/bash
# round 4 GPU call: parity (fast subset) -> A/B base vs product -> short bench -> concurrency probe (last: it may hang)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04a
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "not config4_shape and not full_1gib" > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $O/gpu_tests.txt; exit 1; }
tail -3 $O/gpu_tests.txt
for r in 1 2; do
  for L in lzma-java_amd/build/base/liblzma_mi355x.so lzma-java_amd/build/liblzma_mi355x.so; do
    LZMA_AMD_LIB=$R/$L timeout -k 10 150 python3 tools/ab.py --reps 3 --parity 8 >> $O/ab.jsonl 2>> $O/ab.err || { echo "ab $L failed rc=$?"; tail -5 $O/ab.err; exit 1; }
    tail -1 $O/ab.jsonl | cut -c1-400
  done
done
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --single-stream 16777216 --cpu-sample 0 --parity-streams 64 \
  > $O/bench.json 2> $O/bench.err || { echo "bench failed rc=$?"; tail -20 $O/bench.err; exit 1; }
cut -c1-800 $O/bench.json
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/conc -o conc -- python3 -u $R/tools/concurrency_probe.py \
  > $O/probe.json 2> $O/probe.err
rc=$?
echo "probe rc=$rc"; tail -5 $O/probe.err; cat $O/probe.json
exit 0
