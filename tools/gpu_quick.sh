#!/bin/bash
# Quick GPU iteration: the production-size and fused-op parity tests, the T1
# bench and the row-halo conv stamps.  usage: tools/gpu_quick.sh tag
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-quick}
mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "== $name rc=$rc"; tail -n ${TAILN:-3} $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step tests 300 python -u -m pytest tests/test_production_gpu.py tests/test_fused_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step bench 300 python bench.py --no-cpu-baseline
TAILN=14 step stamps 120 python tools/rows_stamps.py
echo done
