#!/bin/bash
# Pooled-conv kernel check on the GPU box: parity tests of the touched kernel,
# then same-box timings of the new library against abtest/<old>.so.
# usage: tools/gpu_pool1w.sh TAG [old-lib-name] [rows_bench --only list]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; OLD=${2:-old}; ONLY=${3:-pool}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  "tests/test_fused_gpu.py::test_conv_pool_kernels" tests/test_production_gpu.py -k "pool or partial or unpool" > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for L in base $OLD; do
    if [ $L = base ]; then E=""; else E=$PWD/abtest/$L.so; fi
    echo "== $L"
    ACFE_LIB=$E timeout -k 10 200 python tools/rows_bench.py --only $ONLY --iters 9 > $O/rb_${L}_$r.log 2>&1 || { tail -5 $O/rb_${L}_$r.log; exit 1; }
    cat $O/rb_${L}_$r.log
  done
done
echo done
