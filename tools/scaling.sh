#!/bin/bash
# Encoder / decoder time vs streams per CU (256 CUs): 1, 4, 16 streams per CU of 256 KiB.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/scaling
mkdir -p $O
timeout -k 10 300 python3 $R/tools/enc_scaling.py 262144 256,1024,4096 > $O/enc.txt 2>&1 || { echo "enc failed"; tail -5 $O/enc.txt; exit 1; }
cat $O/enc.txt
( for n in 256 1024 4096; do timeout -k 10 200 python3 $R/tools/dec_scaling.py 262144 $n 2 || exit 1; done ) > $O/dec.txt 2>&1 || { echo "dec failed"; tail -5 $O/dec.txt; exit 1; }
cat $O/dec.txt
