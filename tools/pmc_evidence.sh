#!/bin/bash
# Roofline evidence of one workload's dominant kernel, collected inside that
# workload's own bench command: HBM traffic (FETCH_SIZE and WRITE_SIZE, one
# rocprofv3 --pmc pass each) and the SQ counters (two passes), each pass its own
# time limit, the program directly after `--`.  tools/pmc_fold.py then writes
# profiles/pmc_dominant_<key>_<round>.json and profiles/sq_dominant_<key>_<round>.json
# (read by bench.py for roofline.traffic / roofline.counters).
# usage: [SELECT=period:index] tools/pmc_evidence.sh <key> <round> <kernel regex> <algorithmic bytes per launch>
#        <label> <bench args...>   (SELECT: the dominant layer's position among each step's dispatches of the kernel)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
KEY=$1 RND=$2 RX=$3 ALGO=$4 LABEL=$5
shift 5
O=gpurun_out/pmc_${KEY}_${RND}
mkdir -p $O
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES SQ_BUSY_CYCLES"; do
  timeout -s KILL 180 rocprofv3 --pmc $grp --kernel-include-regex "$RX" \
      --output-format csv -d $O/p$i -o pmc -- python bench.py --no-cpu-baseline "$@" > $O/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "pass $i rc=$rc -- stopping"; tail -5 $O/p$i.log; exit $rc
  fi
  i=$((i+1))
done
python tools/pmc_fold.py $O "$RX" "$KEY" "$RND" "$ALGO" "$LABEL" "$*" "$SELECT"
