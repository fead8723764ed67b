#!/bin/bash
# Round 5: GPU suite on the deferred-save build; config-2 bench A/B of DRPO_DEFER_SAVE
# (alternating twice); SAC per-launch timings of both builds.
OUT=gpurun_out/${1:-r05d}
mkdir -p $OUT
export TMPDIR=/tmp
LIBD=$PWD/distributional-reachability-policy-optimization_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > $OUT/pytest.log 2>&1
echo "pytest rc $?" >> $OUT/pytest.log
tail -3 $OUT/pytest.log
line() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); s=d['sac']; k=s['mlp_kernels']
print('$1', 'roll', round(d['roofline']['frac'],4), 'sac', round(s['achieved_tflops_per_gpu'],1), 'TF', ' '.join(f'{n}:{v[\"avg_launch_us\"]}us' for n,v in k.items()), 'fit', round(d['model_fit']['ms_per_fit_step'],4), 'ms')"; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/defer_$i.json 2> $OUT/defer_$i.err || exit 1
  line $OUT/defer_$i.json
  DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_nodefer.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/nodefer_$i.json 2> $OUT/nodefer_$i.err || exit 1
  line $OUT/nodefer_$i.json
done
timeout -k 10 180 python -u profiles/sac_micro.py --steps 10 > $OUT/sac_micro_defer.json 2> $OUT/sac_micro.err || exit 1
DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_nodefer.so timeout -k 10 180 python -u profiles/sac_micro.py --steps 10 > $OUT/sac_micro_nodefer.json 2>> $OUT/sac_micro.err || exit 1
timeout -k 10 300 python -u profiles/shard_fit_probe.py --steps 300 > $OUT/shard_fit_probe.json 2> $OUT/shard_fit_probe.err || exit 1
cat $OUT/shard_fit_probe.json
bash profiles/traffic_elites.sh ${1:-r05d}_te > $OUT/traffic_elites.log 2>&1 || exit 1
cat gpurun_out/${1:-r05d}_te/traffic_e*.json
