#!/bin/bash
# round 4 GPU call 18: where the walk's time goes -- the PosInfo build (build/exp_pi: the walk's
# member inputs gathered in position order by their own kernel, timed apart as mf_posinfo) against
# the product: kernel times (ab.py, BENCH and TEXT) and FETCH_SIZE / WRITE_SIZE of one bench step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04r
mkdir -p $O
cd $R
export TMPDIR=/tmp
X=$R/lzma-java_amd/build/exp_pi/liblzma_mi355x.so
P=$R/lzma-java_amd/build/liblzma_mi355x.so
for r in 1 2; do
  for L in $X $P; do
    LZMA_AMD_LIB=$L timeout -k 10 150 python3 tools/ab.py --reps 2 --parity 4 >> $O/ab.jsonl 2>> $O/ab.err || { echo "ab $L failed rc=$?"; tail -5 $O/ab.err; exit 1; }
    python3 -c "import json; d=[json.loads(l) for l in open('$O/ab.jsonl')][-1]; print(d['lib'][-30:], round(d['MBps'],1), {k: d['kernels_ms'][k] for k in d['kernels_ms'] if k.startswith('mf')}, d['parity'])"
  done
done
for L in $X $P; do
  LZMA_AMD_LIB=$L timeout -k 10 200 python3 tools/ab.py --data text --reps 2 --parity 4 >> $O/ab_text.jsonl 2>> $O/ab.err || { echo "ab text $L failed rc=$?"; tail -5 $O/ab.err; exit 1; }
  python3 -c "import json; d=[json.loads(l) for l in open('$O/ab_text.jsonl')][-1]; print('text', d['lib'][-30:], round(d['MBps'],1), {k: d['kernels_ms'][k] for k in d['kernels_ms'] if k.startswith('mf')}, d['parity'])"
done
cd /tmp
B="$R/bench.py --steps 1 --warmup 0 --cpu-sample 0 --single-stream 0 --no-verify"
for tag in pi prod; do
  L=$P; [ $tag = pi ] && L=$X
  LZMA_AMD_LIB=$L timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d /tmp/f_$tag -o run -- python3 $B > $O/pmc_f_$tag.log 2>&1 || { echo "fetch $tag failed"; exit 1; }
  LZMA_AMD_LIB=$L timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d /tmp/w_$tag -o run -- python3 $B > $O/pmc_w_$tag.log 2>&1 || { echo "write $tag failed"; exit 1; }
  python3 $R/tools/round_reduce.py traffic /tmp/f_$tag /tmp/w_$tag $O/traffic_$tag.json '{"data": "bench"}' > /dev/null || { echo "reduce $tag failed"; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/traffic_$tag.json'))
for k,v in d.items():
  if k.startswith('mf_walk') or k.startswith('mf_posinfo'): print('$tag', k, round(v['fetch_size_bytes_per_launch']/1e9,1), round(v['write_size_bytes_per_launch']/1e9,1))"
done
exit 0
