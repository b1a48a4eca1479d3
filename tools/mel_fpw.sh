cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r02y
for f in 1 2 4 8; do
  ACFE_MEL_FPW=$f timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r02y/bench_$f.log 2>&1 || exit 1
  echo "fpw $f $(grep -o '"avg_launch_ms": [0-9.]*, "GBps": [0-9.]*' gpurun_out/r02y/bench_$f.log | tail -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r02y/bench_$f.log)"
done
