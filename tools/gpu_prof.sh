#!/bin/bash
# rocprofv3 kernel stats of a short bench run.  usage: tools/gpu_prof.sh <tag> [ENV=..]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/prof.log 2>&1 || exit $?
grep '^{' $O/prof.log | head -1 | cut -c1-400
