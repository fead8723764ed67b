#!/bin/bash
# Rollout-phase bounds: library events (default) vs separate torch events around the
# call (DRPO_BENCH_TORCH_PHASE=1); default config-2 bench lines alternating twice.
OUT=gpurun_out/${1:-kt}
mkdir -p $OUT
export TMPDIR=/tmp
line() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$1', round(d['value']/1e6,2), 'M/s frac', round(r['frac'],4), round(r['avg_launch_ms']*1e3,1), 'us', round(d['ms_per_step'],4), 'ms/step sac', round(d['sac']['value'],1))"; }
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > $OUT/lib_$i.json 2> $OUT/lib_$i.err || exit 1
  line $OUT/lib_$i.json
  DRPO_BENCH_TORCH_PHASE=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline > $OUT/torch_$i.json 2> $OUT/torch_$i.err || exit 1
  line $OUT/torch_$i.json
done
timeout -k 10 200 python -u bench.py --no-cpu-baseline --config 5 --steps 5 --warmup 2 > $OUT/c5.json 2> $OUT/c5.err || exit 1
line $OUT/c5.json
