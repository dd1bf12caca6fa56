cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ws; mkdir -p $O
for cfg in "text all" "text 1024,4294967295" "text 0,1023" "text 256,4294967295" "text 0,255" "bench all" "bench 128,4294967295" "bench 0,127"; do
  set -- $cfg
  if [ "$2" = all ]; then timeout -k 10 300 python3 $R/tools/walk_split.py $1 >> $O/ws.jsonl 2>>$O/err.log || exit 1
  else LZG_WALK_ONLY=$2 timeout -k 10 300 python3 $R/tools/walk_split.py $1 >> $O/ws.jsonl 2>>$O/err.log || exit 1; fi
done
cat $O/ws.jsonl
