#!/bin/bash
# HBM traffic of the dominant kernel (stage-1 block-0 3x3 128->128 conv forward,
# T1 shape, batch 512): separate rocprofv3 --pmc passes (never combined with a
# trace domain), each under its own time limit; the first failing pass ends the
# script.  Then tools/pmc_traffic.py writes profiles/pmc_dominant_<tag>.json.
# usage: tools/pmc_traffic.sh [tag]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r01g}
O=gpurun_out/pmc_traffic
mkdir -p $O
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o pmc -- \
      python tools/conv_bench.py --layers 0 --passes fwd --iters 3 > $O/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "pass $i ($grp) rc=$rc -- stopping"; tail -5 $O/p$i.log; exit $rc
  fi
  i=$((i+1))
done
python tools/pmc_traffic.py $O $TAG   # writes profiles/ on the box: rerun locally on the merged gpurun_out/
