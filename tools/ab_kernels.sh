#!/bin/bash
# A/B of two library builds: rocprofv3 kernel stats of a 3-step bench run each.
#   LIBS="pathA pathB" bash tools/ab_kernels.sh   (on the GPU box via gpurun)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for L in $LIBS; do
  LZMA_AMD_LIB=$R/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ab_$i -o run -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-verify > $O/run_$i.log 2>&1 || { echo "run $i failed"; exit 1; }
  python3 $R/tools/round_reduce.py stats /tmp/ab_$i $O/stats_$i.csv || exit 1
  grep '^{' $O/run_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L', 'value', round(d['value'],1))"
  head -8 $O/stats_$i.csv
  i=$((i+1))
done
