#!/bin/bash
# T1 bench + rocprofv3 kernel stats of the same command.  usage: tools/gpu_benchprof.sh tag
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-bp}
mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
tail -c 600 $O/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/prof.log 2>&1 || exit $?
python tools/prof_summary.py $O/prof/run_kernel_stats.csv $O/prof/run_kernel_trace.csv 13 > $O/summary.md 2>&1; head -40 $O/summary.md
