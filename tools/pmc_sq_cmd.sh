#!/bin/bash
# tools/pmc_sq.sh's two SQ counter passes over any python tool instead of the
# T1 bench (one rocprofv3 --pmc pass per group, each its own time limit; the
# interpreter follows `--` directly).
# usage: tools/pmc_sq_cmd.sh <tag> <kernel regex> <script.py> [args...]   output: gpurun_out/pmc_<tag>/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1 RX=$2
shift 2
O=gpurun_out/pmc_$TAG
mkdir -p $O
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES SQ_BUSY_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$RX" \
      --output-format csv -d $O/p$i -o pmc -- python "$@" > $O/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "pass $i rc=$rc -- stopping"; tail -5 $O/p$i.log; exit $rc
  fi
  i=$((i+1))
done
echo pmc done
