#!/bin/bash
# SQ / GRBM counters (MFMA busy, CU busy, wait / stall split, LDS) of chosen
# kernels inside the T1 bench, one rocprofv3 --pmc pass per group, each pass its
# own time limit.  The program follows `--` directly (no wrapper).
# usage: tools/pmc_sq.sh <tag> [kernel regex]    output: gpurun_out/pmc_<tag>/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-sq}
RX=${2:-k_conv3x3_rows<128, 4, [12], true|k_wgrad3x3_halo<128, true>}
O=gpurun_out/pmc_$TAG
mkdir -p $O
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES SQ_BUSY_CYCLES"; do
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$RX" \
      --output-format csv -d $O/p$i -o pmc -- python bench.py --no-cpu-baseline --no-extra --steps 2 --warmup 1 ${BENCH_ARGS:-} > $O/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "pass $i rc=$rc -- stopping"; tail -5 $O/p$i.log; exit $rc
  fi
  i=$((i+1))
done
echo pmc done
