#!/bin/bash
# Round-2 measurement session: entry points (config P, spectrogram / raw
# training), the front-end tests, the e2e TFRecord line, wr_resnet training,
# fp32 streaming, inference, the CPU baseline suite.  Each step has its own
# limit; the first failure ends the script.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r02g}; mkdir -p $O
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 $O/$name.log | cut -c1-700; [ $rc -eq 0 ] || exit $rc; }
run entry 400 python -u -m pytest tests/test_entrypoints.py tests/test_frontend_gpu.py -m gpu -x -v -s --timeout 300 --timeout-method thread
grep "config P" $O/entry.log
run e2e 300 python bench.py --workload e2e --steps 12 --warmup 2
run wrn 300 python bench.py --model wrn --classes 2 --no-cpu-baseline
run stream32 300 python bench.py --workload stream --dtype fp32 --steps 3 --warmup 1
run infer 300 python bench.py --workload infer --steps 5 --warmup 2
[ -n "$SKIP_CPU" ] || run cpu 900 python tools/cpu_baseline.py --out $O/cpu_baseline.json
echo all done
