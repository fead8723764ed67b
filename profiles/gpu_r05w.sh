#!/bin/bash
# Round 5: rollout A/B builds (ring depth scale 16 / 8 vs 12, member-L1 prefetch, actor
# biases in LDS): config-2 rollout-only bench lines, three alternating rounds.
OUT=gpurun_out/${1:-r05w}
mkdir -p $OUT
export TMPDIR=/tmp
LIBD=$PWD/distributional-reachability-policy-optimization_amd
line() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', round(d['value']/1e6,1), 'M/s frac', round(r['frac'],4), round(r['avg_launch_ms']*1e3,1), 'us')"; }
for i in 1 2 3; do
  for t in base pf16 m1 abias; do
    if [ $t = base ]; then L=""; else L="DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_$t.so"; fi
    env $L timeout -k 10 200 python -u bench.py --no-cpu-baseline --rollout-only > $OUT/c2_$t.json 2> $OUT/c2_$t.err || exit 1
    line $OUT/c2_$t.json $t
  done
done
