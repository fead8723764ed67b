#!/bin/bash
# Whole-bench A/B by environment switch ($2=$3 vs default): GPU suite (default), then
# config-2 bench lines (rollout + SAC + fit) alternating twice. Usage:
#   bash profiles/gpu_bench_ab.sh <tag> <ENV_VAR> <value>
OUT=gpurun_out/${1:-bab}
V=$2; X=$3
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
line() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); s=d['sac']; k=s['mlp_kernels']
print('$1', 'roll', round(d['roofline']['frac'],4), 'sac', round(s['achieved_tflops_per_gpu'],1), 'TF', ' '.join(f'{n}:{v[\"avg_launch_us\"]}us' for n,v in k.items()), 'fit', round(d['model_fit']['ms_per_fit_step'],4), 'ms')"; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/def_$i.json 2> $OUT/def_$i.err || exit 1
  line $OUT/def_$i.json
  env $V=$X timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/alt_$i.json 2> $OUT/alt_$i.err || exit 1
  line $OUT/alt_$i.json
done
