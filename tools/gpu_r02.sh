#!/bin/bash
# Round-2 GPU session: all -m gpu tests, smoke, a 2-rank data-parallel
# rehearsal on the one GPU (gloo backend: RCCL needs one GPU per rank), the
# driver's default bench line.  Each step has its own limit; the first failure
# ends the script.   usage: tools/gpu_r02.sh <tag> [tests|dp|bench|prof ...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r02}; shift
STEPS=${*:-tests dp bench}
O=gpurun_out/$TAG
mkdir -p $O
step() { # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -5 $O/$name.log
  [ $rc -eq 0 ] || exit $rc
}
for s in $STEPS; do
  case $s in
    tests) step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
           step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    ptests) step ptests 600 python -u -m pytest ${PTESTS:-tests/test_production_gpu.py} -m gpu -x -v --timeout 120 --timeout-method thread ;;
    dp) ACFE_DIST_BACKEND=gloo step dp 300 python bench.py --gpus 2 --steps 3 --warmup 2 --batch 64 --no-cpu-baseline ;;
    bench) step bench 600 python bench.py ${BENCH_ARGS:-} ;;
    prof) step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
            python bench.py --no-cpu-baseline --steps 10 --warmup 3 ${BENCH_ARGS:-} ;;
  esac
done
echo done
