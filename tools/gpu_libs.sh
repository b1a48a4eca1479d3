#!/bin/bash
# Same-box timings of library variants with tools/rows_bench.py (no parity
# tests: timing-only variants may compute wrong values).
# usage: tools/gpu_libs.sh TAG ONLY lib1 lib2 ...   ("base" = the in-tree build)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; ONLY=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
for r in 1 2; do
  for L in "$@"; do
    if [ $L = base ]; then E=""; else E=$PWD/abtest/$L.so; fi
    ACFE_LIB=$E timeout -k 10 200 python tools/rows_bench.py --only $ONLY --iters 9 > $O/rb_${L}_$r.log 2>&1 || { tail -5 $O/rb_${L}_$r.log; exit 1; }
    echo "$L $(grep -v amdgpu.ids $O/rb_${L}_$r.log | tr -s ' ' | tr '\n' ' ')"
  done
done
echo done
