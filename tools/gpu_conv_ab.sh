#!/bin/bash
# Conv kernel iteration: GPU conv parity tests, then the T1 conv microbench with
# the pipelined kernel and (A/B) the 2-stage kernel.  usage: tools/gpu_conv_ab.sh [tag] [pytest -k expr]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-conv}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_fused_gpu.py -x -q --timeout 300 --timeout-method thread ${2:+-k "$2"} > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/conv_bench.py --iters 5 > $O/bench_pipe.log 2>&1 || { tail $O/bench_pipe.log; exit 1; }
cat $O/bench_pipe.log
ACFE_CONV_NO_PIPE=1 timeout -k 10 300 python tools/conv_bench.py --iters 5 --passes fwd,dgrad > $O/bench_old.log 2>&1 || { tail $O/bench_old.log; exit 1; }
cat $O/bench_old.log
