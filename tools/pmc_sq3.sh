#!/bin/bash
# Instruction-mix counters (SALU / branch / per-category active cycles) of the
# chosen kernels inside a bench run: one rocprofv3 --pmc pass, its own limit.
# usage: BENCH_ARGS='--model wrn --classes 2' tools/pmc_sq3.sh <tag> <kernel regex>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-sq3}
RX=${2:-k_conv3x3_r64}
O=gpurun_out/pmc_$TAG
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA \
    SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_WAVES --kernel-include-regex "$RX" \
    --output-format csv -d $O/p2 -o pmc -- python bench.py --no-cpu-baseline --no-extra --steps 2 --warmup 1 ${BENCH_ARGS:-} \
    > $O/p2.log 2>&1
rc=$?
[ $rc -ne 0 ] && { echo "pass rc=$rc"; tail -5 $O/p2.log; exit $rc; }
echo pmc done
