#!/bin/bash
# Build variants of libacfe.so with extra compile flags into abtest/<name>.so
# (CPU side, here), or time them on the GPU box with tools/rows_bench.py.
#   tools/ab_lib.sh build <name> "<-D flags>"
#   tools/ab_lib.sh run <tag> "<rows_bench args>" name1 name2 ...   (on the box; "base" = the in-tree build)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
case $1 in
  build)
    name=$2; flags=$3
    out=$ROOT/abtest/$name; mkdir -p $out
    cd $ROOT/audio-training_amd/csrc
    for f in *.hip; do
      extra=""; { [ $f = pool1w.hip ] || [ $f = frontend.hip ] || [ $f = rows64.hip ]; } && extra=-fno-slp-vectorize
      /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -DACFE_ABLATE $flags $extra -c $f -o $out/${f%.hip}.o &
    done
    wait
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $ROOT/abtest/$name.so $out/*.o
    rm -rf $out
    echo built abtest/$name.so ;;
  run)
    cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
    tag=$2; args=$3; shift 3
    O=gpurun_out/$tag; mkdir -p $O
    for name in "$@"; do
      if [ "$name" = base ]; then lib=""; else lib=$PWD/abtest/$name.so; fi
      echo "== $name"
      ACFE_LIB=$lib timeout -k 10 240 python tools/rows_bench.py $args > $O/$name.log 2>&1 || { tail -5 $O/$name.log; exit 1; }
      cat $O/$name.log
    done ;;
esac
