#!/bin/bash
# A/B of the wgrad BN-backward fold's transform position (ACFE_FB_MID builds
# in abtest/, tools/ab_lib.sh) with tools/fold_bench.py at the wr_resnet and
# wr_resnet_bird stage-1 shapes.  usage (on the box): tools/fold_ab.sh v1 v2 ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  for shp in "512 128 513 64 64" "512 64 128 64 64"; do
    echo "== fbmid$v $shp"
    ACFE_LIB=$PWD/abtest/fbmid$v.so timeout -k 10 120 python tools/fold_bench.py $shp 10 ${RATE:-0.1} || exit 1
  done
done
