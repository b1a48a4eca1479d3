cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r01d
timeout -k 10 300 python bench.py --workload infer --steps 10 --warmup 3 > gpurun_out/r01d/infer.log 2>&1 || { tail gpurun_out/r01d/infer.log; exit 1; }
tail -1 gpurun_out/r01d/infer.log
timeout -k 10 300 python bench.py --workload stream --steps 3 --warmup 1 > gpurun_out/r01d/stream.log 2>&1 || { tail gpurun_out/r01d/stream.log; exit 1; }
tail -1 gpurun_out/r01d/stream.log
bash tools/pmc_traffic.sh r01
