cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r02aa; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_production_gpu.py tests/test_fused_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for t in 5 6; do
  ACFE_ROWS64_TR=$t timeout -k 10 240 python tools/rows_bench.py --only add,drop64 --iters 9 > $O/rows_$t.log 2>&1 || exit 1
  ACFE_ROWS64_TR=$t timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_$t.log 2>&1 || exit 1
  echo "TR $t $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$t.log)"; grep -v amdgpu.ids $O/rows_$t.log
done
