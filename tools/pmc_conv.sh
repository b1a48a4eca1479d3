#!/bin/bash
# PMC passes over the T1 conv microbench (one counter group per rocprofv3 run,
# --pmc never combined with trace domains).  The first pass that fails for any
# reason ends the script, so nothing more runs on the GPU after it.
# Output: gpurun_out/pmc_conv/p<i>/   usage: tools/pmc_conv.sh [layer indices]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc_conv
L=${1:-0}
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
           "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_conv/p$i -o pmc -- \
      python tools/conv_bench.py --layers "$L" --passes "${PASSES:-fwd,dgrad,wgrad}" --iters 2 > gpurun_out/pmc_conv/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "pass $i ($grp) rc=$rc -- stopping"
    tail -5 gpurun_out/pmc_conv/p$i.log
    exit $rc
  fi
  i=$((i+1))
done
