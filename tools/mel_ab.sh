cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r02x
timeout -k 10 300 python -u -m pytest tests/test_frontend_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02x/tests.log 2>&1 || { tail -20 gpurun_out/r02x/tests.log; exit 1; }
tail -2 gpurun_out/r02x/tests.log
for v in w2 w1; do
  if [ $v = w1 ]; then E="ACFE_MEL_W1=1"; L=""; elif [ $v = w4 ]; then E="ACFE_MEL_W1=0"; L=$PWD/abtest/melw4.so; else E="ACFE_MEL_W1=0"; L=""; fi
  env $E ACFE_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r02x/bench_$v.log 2>&1 || exit 1
  echo "$v $(grep -o '"mel_pipeline": {[^}]*}' gpurun_out/r02x/bench_$v.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r02x/bench_$v.log)"
done
