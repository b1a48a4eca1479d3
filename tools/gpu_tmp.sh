cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for f in "" "--no-stats" "--no-bias" "--no-stats --no-bias"; do
  echo "== $f"; timeout -k 10 120 python tools/conv_bench.py --layers 0,5 --passes fwd --iters 5 $f 2>&1 | grep -v amdgpu.ids || exit 1
done
