#!/bin/bash
# Round 5: GPU suite (pair / chain multi-job forwards), bench line, SAC per-launch timings,
# member-shard fit probe.
OUT=gpurun_out/${1:-r05g}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > $OUT/pytest.log 2>&1
echo "pytest rc $?" >> $OUT/pytest.log
tail -3 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
python -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); s=d['sac']; k=s['mlp_kernels']
print('value', round(d['value']/1e6,1), 'roll', round(d['roofline']['frac'],4), 'sac', round(s['achieved_tflops_per_gpu'],2), 'TF', s['value'], ' '.join(f'{n}:{v[\"avg_launch_us\"]}us/{v[\"launches\"]}' for n,v in k.items()), 'fit', d['model_fit']['ms_per_fit_step'])"
timeout -k 10 180 python -u profiles/sac_micro.py --steps 10 > $OUT/sac_micro.json 2> $OUT/sac_micro.err || exit 1
timeout -k 10 300 python -u profiles/shard_fit_probe.py --steps 300 > $OUT/shard_fit_probe.json 2> $OUT/shard_fit_probe.err || exit 1
cat $OUT/shard_fit_probe.json
