#!/bin/bash
# Round 5: GPU suite on the swizzled-store build, the layer probe (swizzled / plain stores),
# and a config-2 bench A/B of the epilogue store swizzle (DRPO_LDS_SWZ) alternating twice.
OUT=gpurun_out/${1:-r05b}
mkdir -p $OUT
export TMPDIR=/tmp
LIBD=$PWD/distributional-reachability-policy-optimization_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > $OUT/pytest.log 2>&1
echo "pytest rc $?" >> $OUT/pytest.log
tail -3 $OUT/pytest.log
timeout -k 10 120 ./profiles/layer_probe > $OUT/layer_probe.txt 2>&1 || exit 1
timeout -k 10 120 ./profiles/layer_probe_noswz > $OUT/layer_probe_noswz.txt 2>&1 || exit 1
cat $OUT/layer_probe.txt $OUT/layer_probe_noswz.txt
line() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); s=d['sac']; k=s['mlp_kernels']
print('$1', 'roll', round(d['roofline']['frac'],4), 'sac', round(s['achieved_tflops_per_gpu'],1), 'TF', ' '.join(f'{n}:{v[\"avg_launch_us\"]}us' for n,v in k.items()), 'fit', round(d['model_fit']['ms_per_fit_step'],4), 'ms')"; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/swz_$i.json 2> $OUT/swz_$i.err || exit 1
  line $OUT/swz_$i.json
  DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_noswz.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/noswz_$i.json 2> $OUT/noswz_$i.err || exit 1
  line $OUT/noswz_$i.json
done
