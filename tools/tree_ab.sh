# Same-box A/B of the T1 bench line: the working tree ("new") against a copy
# of an earlier commit's tree with its own built library in abtest/oldtree
# ("old").  usage (on the box): bash tools/tree_ab.sh <tag> [rounds]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-ab}; n=${2:-3}
O=gpurun_out/$tag; mkdir -p $O
for i in $(seq $n); do
  for v in new old; do
    if [ $v = old ]; then b=abtest/oldtree/bench.py; else b=bench.py; fi
    timeout -k 10 300 python -u $b --steps 20 --warmup 5 --no-cpu-baseline > $O/b_${v}_$i.json 2>$O/b_${v}_$i.err || exit 1
    python -c "import json,sys; d=json.loads(open('$O/b_${v}_$i.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
  done
done
