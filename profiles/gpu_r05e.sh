#!/bin/bash
# Round 5: GPU suite (default build: Pre0 + tile head), SAC forward stamps, and a config-2
# bench A/B over the forward variants, alternating twice:
#   default (Pre0 + head tile), nopre0 (head tile only), nohead (Pre0 only), base (neither)
OUT=gpurun_out/${1:-r05e}
mkdir -p $OUT
export TMPDIR=/tmp
LIBD=$PWD/distributional-reachability-policy-optimization_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > $OUT/pytest.log 2>&1
echo "pytest rc $?" >> $OUT/pytest.log
tail -3 $OUT/pytest.log
DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_stamps.so timeout -k 10 180 python -u profiles/sac_fwd_stamps.py > $OUT/sac_fwd_stamps.txt 2> $OUT/sac_fwd_stamps.err || { tail $OUT/sac_fwd_stamps.err; exit 1; }
cat $OUT/sac_fwd_stamps.txt
line() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); s=d['sac']; k=s['mlp_kernels']
print('$1', 'roll', round(d['roofline']['frac'],4), 'sac', round(s['achieved_tflops_per_gpu'],1), 'TF', ' '.join(f'{n}:{v[\"avg_launch_us\"]}us' for n,v in k.items()), 'fit', round(d['model_fit']['ms_per_fit_step'],4), 'ms')"; }
for i in 1 2; do
  for v in default nopre0 nohead base; do
    if [ $v = default ]; then L=""; else L=$LIBD/libdrpo_hip_$v.so; fi
    DRPO_LIB_OVERRIDE=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-fit > $OUT/${v}_$i.json 2> $OUT/${v}_$i.err || exit 1
    line $OUT/${v}_$i.json
  done
done
