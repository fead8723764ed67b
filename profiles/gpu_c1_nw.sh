#!/bin/bash
# Config 1 (B=256: 16 row tiles on 256 CUs) rollout with 8- vs 16-wave workgroups
# (DRPO_ROLLOUT_NW=16), rollout-only lines alternating twice.
OUT=gpurun_out/${1:-c1nw}
mkdir -p $OUT
export TMPDIR=/tmp
line() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$1', round(d['value']/1e6,2), 'M/s frac', round(r['frac'],4), round(r['avg_launch_ms']*1e3,1), 'us')"; }
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --rollout-only --config 1 > $OUT/nw8_$i.json 2> $OUT/nw8_$i.err || exit 1
  line $OUT/nw8_$i.json
  DRPO_ROLLOUT_NW=16 timeout -k 10 200 python -u bench.py --no-cpu-baseline --rollout-only --config 1 > $OUT/nw16_$i.json 2> $OUT/nw16_$i.err || exit 1
  line $OUT/nw16_$i.json
done
