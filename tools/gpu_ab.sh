#!/bin/bash
# A/B on the GPU box: parity tests of the touched area, then the T1 bench with
# and without an env switch.  usage: tools/gpu_ab.sh <tag> <tests> <ENV=1>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; TESTS=$2; SW=$3
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_new.log 2>&1 || exit $?
env $SW timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_old.log 2>&1 || exit $?
python - $O <<'PY'
import json, sys
for k in ("new", "old"):
    l = [x for x in open(f"{sys.argv[1]}/bench_{k}.log") if x.startswith("{")][0]
    d = json.loads(l)
    print(k, d["value"], d["ms_per_step"], "mel", d["mel_pipeline"]["avg_launch_ms"])
PY
