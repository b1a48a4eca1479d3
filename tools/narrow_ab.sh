# A/B of k_conv3x3_narrow with 4 vs 8 waves per workgroup (ACFE_NARROW_WAVES):
# parity tests under both, then per-layer timing and the T1 bench line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for nw in 8 4; do
  ACFE_NARROW_WAVES=$nw timeout -k 10 300 python -u -m pytest tests/test_production_gpu.py -x -q -k "narrow" --timeout 120 --timeout-method thread > gpurun_out/narrow_t$nw.log 2>&1; rc=$?; tail -2 gpurun_out/narrow_t$nw.log; [ $rc -eq 0 ] || exit $rc
done
for nw in 8 4; do
  echo "== waves $nw"
  ACFE_NARROW_WAVES=$nw timeout -k 10 300 python -u tools/layer_profile.py > gpurun_out/narrow_lp$nw.log 2>&1 || exit 1
  grep -i "narrow\|32, 64\|16, 32\|total" gpurun_out/narrow_lp$nw.log | head -30
done
for nw in 8 4 8 4; do
  ACFE_NARROW_WAVES=$nw timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/narrow_b$nw.json 2>gpurun_out/narrow_b$nw.err || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/narrow_b$nw.json').read().strip().splitlines()[-1]); print('waves $nw', d['value'], d['ms_per_step'])"
done
