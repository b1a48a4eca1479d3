#!/bin/bash
# A/B of halo-wgrad library variants (abtest/<name>.so, tools/ab_lib.sh) with
# tools/wgrad_bench.py at the wr_resnet / wr_resnet_bird layer shapes.
# usage (on the box): tools/wg_ab.sh name1 name2 ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  for shp in "512 128 513 64 64" "512 64 128 64 64" "512 64 257 128 128" "512 22 86 256 256" "512 128 256 128 128 10 unpool"; do
    ACFE_LIB=$PWD/abtest/$v.so timeout -k 10 120 python tools/wgrad_bench.py $shp 10 | sed "s/^/$v /" || exit 1
  done
done
