#!/bin/bash
# Round-5 evidence on the final build, part B: bench lines for configs 1-5 (config 2 with
# the CPU baseline; traffic attached from the digest-stamped JSONs in profiles/) and the
# default bench line (no flags).
OUT=gpurun_out/${1:-r05final}
mkdir -p $OUT
export TMPDIR=/tmp
bash profiles/bench_configs.sh ${1:-r05final} 1 2 3 4 5 || exit 1
timeout -k 10 400 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
for f in $OUT/bench_c*.json $OUT/bench_default.json; do
  python -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); s=d.get('sac',{}); r=d['roofline']
print('$f'.split('/')[-1], round(d['value']/1e6,1), 'roll', round(r['frac'],4), 'traffic', r.get('traffic'), 'sac', s.get('achieved_tflops_per_gpu'), 'fit', d.get('model_fit',{}).get('ms_per_fit_step'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))"
done
