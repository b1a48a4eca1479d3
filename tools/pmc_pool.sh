#!/bin/bash
# HBM traffic (rocprofv3 --pmc, one counter group per pass, kernel-filtered) of
# the bench's dominant kernel: the stage-1 block-0 3x3 128->128 conv forward with
# the 2x2 max-pool epilogue (k_conv3x3_1w<1, 2, true>: one wave per SIMD,
# chunk-resident 4-row tiles), inside the T1 bench.  Then tools/pmc_traffic.py folds the passes into
# profiles/pmc_dominant_<tag>.json.
# usage: tools/pmc_pool.sh [tag] [kernel regex]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r02}
RX=${2:-k_conv3x3_1w<1}
O=gpurun_out/pmc_pool
mkdir -p $O
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 180 rocprofv3 --pmc $grp --kernel-include-regex "$RX" \
      --output-format csv -d $O/p$i -o pmc -- python bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "pass $i ($grp) rc=$rc -- stopping"; tail -5 $O/p$i.log; exit $rc
  fi
  i=$((i+1))
done
KNAME="${RX%%<*}" python tools/pmc_traffic.py $O $TAG pool
