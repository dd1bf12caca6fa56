#!/bin/bash
# Round-3 measurement call: the default bench line (with single_stream and the CPU thread
# sweep), then the rocprof kernel stats / PMC traffic / issue counters of the bench
# workload and of config 3 (TEXT, dict 2^28). Each step has its own time limit.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03
mkdir -p $O
for s in ${*:-bench prof text}; do
  case $s in
    bench) (cd $R && timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err) || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 1; }
           cat $O/bench.json ;;
    prof|text) bash $R/tools/profile_r03.sh $s || exit 1 ;;
  esac
done
