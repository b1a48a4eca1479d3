cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 300 --timeout-method thread -k "conv" > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/layer_profile.py 2>&1 | tail -3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rd -o run -- python tools/conv_bench.py --iters 3 --passes wgrad > gpurun_out/rd.log 2>&1; echo rc=$?
