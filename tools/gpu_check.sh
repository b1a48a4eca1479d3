#!/bin/bash
# One GPU-box session: GPU parity tests, smoke, bench, rocprofv3 kernel-trace
# summary of the same bench command.  Each GPU step has its own time limit;
# the first failing step ends the script (nothing more touches the GPU).
# usage: tools/gpu_check.sh [tag]       output: gpurun_out/<tag>/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-run}
O=gpurun_out/$TAG
mkdir -p $O
set -o pipefail
step() { # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -4 $O/$name.log
  [ $rc -eq 0 ] || exit $rc
}
if [ -z "$SKIP_TESTS" ]; then
  step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench 600 python bench.py ${BENCH_ARGS:-}
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python bench.py --no-cpu-baseline --steps 10 --warmup 3 ${BENCH_ARGS:-}
echo done
