#!/bin/bash
# Build the product library in a staging directory and move it into place with one
# rename, so a gpurun snapshot taken meanwhile never holds a half-written .so.
# usage: tools/build_atomic.sh [DEST_DIR (default lzma-java_amd/build)] [extra HIPFLAGS]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
DEST=${1:-$R/lzma-java_amd/build}
EXTRA=${2:-}
STAGE=$R/lzma-java_amd/.stage_$(basename $DEST)
make -s -j8 -C $R/lzma-java_amd OUT=$STAGE HIPFLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function -Wno-unused-variable -Wno-unused-value -Wno-unused-result $EXTRA"
mkdir -p $DEST
cp $STAGE/liblzma_mi355x.so $DEST/.liblzma_mi355x.so.tmp
mv $DEST/.liblzma_mi355x.so.tmp $DEST/liblzma_mi355x.so
echo "built $DEST/liblzma_mi355x.so"
