cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_fused_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
for tr in 6 3; do
echo "== TR $tr"
ACFE_CONV_ROWS_TR=$tr timeout -k 10 300 python tools/conv_bench.py --iters 5 --layers 0,2,3 --passes fwd,dgrad 2>&1 | grep -v amdgpu.ids || exit 1
done
