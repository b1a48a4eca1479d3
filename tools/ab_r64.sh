#!/bin/bash
# Stamps-build variants of rows64.hip only, linked with the other stamps
# objects (make -C audio-training_amd/csrc stamps first): abtest/<name>.so
#   tools/ab_r64.sh <name> "<-D flags>"
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; flags=$2
cd $ROOT/audio-training_amd/csrc
mkdir -p $ROOT/abtest/$name
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -fno-slp-vectorize -DACFE_ROWS_STAMPS \
  -DACFE_P1W_STAMPS -DACFE_R64_STAMPS $flags -c rows64.hip -o $ROOT/abtest/$name/rows64.o
objs=$(ls build_stamps/*.o | grep -v rows64.o)
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $ROOT/abtest/$name.so $objs $ROOT/abtest/$name/rows64.o -lz -ldl
rm -rf $ROOT/abtest/$name
echo built abtest/$name.so
