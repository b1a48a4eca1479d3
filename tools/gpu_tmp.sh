cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_fused_gpu.py tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -15 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/conv_bench.py --iters 5 --layers 1 2>&1 | grep -v amdgpu.ids || exit 1
ACFE_CONV_NO_1X1=1 timeout -k 10 300 python tools/conv_bench.py --iters 5 --layers 1 --passes fwd,dgrad 2>&1 | grep -v amdgpu.ids
