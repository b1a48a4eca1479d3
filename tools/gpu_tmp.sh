cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/xres
timeout -k 10 300 python -u tools/layer_profile.py > gpurun_out/xres/lp.log 2>&1 || exit 1
cat gpurun_out/xres/lp.log | grep -v amdgpu.ids
for v in new old new old; do
  if [ $v = old ]; then lib=$PWD/abtest/old.so; else lib=""; fi
  ACFE_LIB=$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/xres/b_$v.json 2>gpurun_out/xres/b_$v.err || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/xres/b_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done
