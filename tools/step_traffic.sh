#!/bin/bash
# HBM traffic of every kernel of a training step: rocprofv3 --pmc FETCH_SIZE
# and WRITE_SIZE in two separate passes (never combined with a trace domain),
# each under its own time limit, over a short bench run; then
# tools/step_traffic.py folds them into a per-kernel table (GB per step).
# usage: tools/step_traffic.sh <tag> <bench args...>   (e.g. wrn_r05 --model wrn --classes 2)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1
shift
O=gpurun_out/step_traffic_$TAG
mkdir -p $O
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o pmc -- \
      python bench.py --no-cpu-baseline --no-extra --steps 2 --warmup 1 "$@" > $O/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "pass $i ($grp) rc=$rc -- stopping"; tail -5 $O/p$i.log; exit $rc
  fi
  i=$((i+1))
done
python tools/step_traffic.py $O "$TAG" "$*"
