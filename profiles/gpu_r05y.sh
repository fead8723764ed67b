#!/bin/bash
# Round 5: deferred coalesced forward saves (DRPO_DEFER_SAVES) + member-L1 prefetch
# (DRPO_PREFETCH_M1): GPU suite on the default build, then SAC per-launch A/B and
# rollout-only A/B, alternating.
OUT=gpurun_out/${1:-r05y}
mkdir -p $OUT
export TMPDIR=/tmp
LIBD=$PWD/distributional-reachability-policy-optimization_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc $rc" >> $OUT/pytest.log; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit 1
line() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', round(d['value']/1e6,1), 'M/s frac', round(r['frac'],4), round(r['avg_launch_ms']*1e3,1), 'us')"; }
for i in 1 2; do
  for t in base nodefer; do
    if [ $t = base ]; then L=""; else L="DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_$t.so"; fi
    env $L timeout -k 10 180 python -u profiles/sac_micro.py --steps 10 > $OUT/sac_$t.json 2> $OUT/sac_$t.err || exit 1
    python - $OUT/sac_$t.json $t <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], ' '.join(f"{k}:{v['avg_ms']*1e3:.1f}" for k, v in d.items() if isinstance(v, dict) and 'avg_ms' in v and k.startswith('mlp_fwd')))
PY
  done
  for t in base nom1; do
    if [ $t = base ]; then L=""; else L="DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_$t.so"; fi
    env $L timeout -k 10 200 python -u bench.py --no-cpu-baseline --rollout-only > $OUT/c2_$t.json 2> $OUT/c2_$t.err || exit 1
    line $OUT/c2_$t.json $t
  done
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
python -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); s=d['sac']
print('value', round(d['value']/1e6,1), 'roll', round(d['roofline']['frac'],4), 'sac', round(s['achieved_tflops_per_gpu'],2), 'fit', d['model_fit']['ms_per_fit_step'])"
