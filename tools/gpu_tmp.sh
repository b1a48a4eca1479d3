cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pro2
for i in 1 2; do
for v in "1 1" "0 1" "1 0" "0 0"; do
  set -- $v
  ACFE_BN_PROLOGUE_POOL=$1 ACFE_BN_PROLOGUE_C1=$2 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/pro2/b.json 2>gpurun_out/pro2/b.err || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/pro2/b.json').read().strip().splitlines()[-1]); print('pool $1 c1 $2', d['value'], d['ms_per_step'])"
done
done
