#!/bin/bash
# Rollout-kernel iteration: rollout parity tests, config-2 stamps, rollout-only bench
# lines at configs 2 (twice), 3 and 4. Usage: bash profiles/gpu_roll_iter.sh <tag>
OUT=gpurun_out/${1:-ri}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_configs.py tests/test_gpu_trainer.py -m gpu -x -q --timeout 200 --timeout-method thread -rf > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
STAMPS=$PWD/distributional-reachability-policy-optimization_amd/libdrpo_hip_stamps.so
DRPO_LIB_OVERRIDE=$STAMPS DRPO_STAMPS_CONFIG=2 DRPO_STAMPS_ROLLOUT=fused timeout -k 10 120 python profiles/stamps.py > $OUT/stamps_c2.txt 2>&1 || exit 1
for c in 2 2 3 4; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --rollout-only --config $c > $OUT/c$c.json 2> $OUT/c$c.err || exit 1
  python -c "import json; d=json.loads(open('$OUT/c$c.json').read().strip().splitlines()[-1]); r=d['roofline']; print('config $c', round(d['value']/1e6,1), 'M/s frac', round(r['frac'],4), round(r['avg_launch_ms']*1e3,1), 'us')"
done
cat $OUT/stamps_c2.txt
