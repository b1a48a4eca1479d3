#!/bin/bash
# Generic PMC passes: tools/pmc_groups.sh <outdir-tag> "<cmd>" "<group1>" "<group2>" ...
# one rocprofv3 --pmc run per group (never combined with a trace domain), each
# under its own hard time limit; the first failing pass stops the script.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; CMD=$2; shift 2
O=gpurun_out/pmc_$TAG
mkdir -p $O
i=0
for grp in "$@"; do
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o pmc -- $CMD > $O/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i ($grp) rc=$rc -- stopping"; tail -5 $O/p$i.log; exit $rc; fi
  i=$((i+1))
done
echo ok
