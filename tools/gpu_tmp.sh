cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pro
timeout -k 10 300 python -u -m pytest tests/test_production_gpu.py -x -q -k "prologue" --timeout 120 --timeout-method thread > gpurun_out/pro/t1.log 2>&1; rc=$?; tail -30 gpurun_out/pro/t1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_production_gpu.py tests/test_model_gpu.py tests/test_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pro/t2.log 2>&1; rc=$?; tail -5 gpurun_out/pro/t2.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  ACFE_BN_PROLOGUE=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/pro/b_$v.json 2>gpurun_out/pro/b_$v.err || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/pro/b_$v.json').read().strip().splitlines()[-1]); print('pro $v', d['value'], d['ms_per_step'])"
done
