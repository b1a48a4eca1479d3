cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r02ae; mkdir -p $O
for v in base melpf2 melpf3; do
  if [ $v = base ]; then L=""; else L=$PWD/abtest/$v.so; fi
  ACFE_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_frontend_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1 || { tail -5 $O/tests_$v.log; exit 1; }
  ACFE_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_$v.log 2>&1 || exit 1
  echo "$v $(tail -1 $O/tests_$v.log) $(grep -o '"avg_launch_ms": [0-9.]*, "GBps": [0-9.]*' $O/bench_$v.log | tail -1) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$v.log)"
done
