#!/bin/bash
# Rollout A/B by environment switch: rollout parity tests (default build), config-2 stamps
# and rollout-only bench lines for the default and with $2=1 (two alternating rounds),
# config 3 once each. Usage: bash profiles/gpu_roll_ab.sh <tag> <ENV_VAR>
OUT=gpurun_out/${1:-rab}
V=$2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_configs.py tests/test_gpu_trainer.py -m gpu -x -q --timeout 200 --timeout-method thread -rf > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
STAMPS=$PWD/distributional-reachability-policy-optimization_amd/libdrpo_hip_stamps.so
DRPO_LIB_OVERRIDE=$STAMPS DRPO_STAMPS_CONFIG=2 DRPO_STAMPS_ROLLOUT=fused timeout -k 10 120 python profiles/stamps.py > $OUT/stamps_on.txt 2>&1 || exit 1
env $V=1 DRPO_LIB_OVERRIDE=$STAMPS DRPO_STAMPS_CONFIG=2 DRPO_STAMPS_ROLLOUT=fused timeout -k 10 120 python profiles/stamps.py > $OUT/stamps_off.txt 2>&1 || exit 1
line() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$1', round(d['value']/1e6,1), 'M/s frac', round(r['frac'],4), round(r['avg_launch_ms']*1e3,1), 'us')"; }
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --rollout-only > $OUT/c2_on_$i.json 2> $OUT/c2_on_$i.err || exit 1
  line $OUT/c2_on_$i.json
  env $V=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --rollout-only > $OUT/c2_off_$i.json 2> $OUT/c2_off_$i.err || exit 1
  line $OUT/c2_off_$i.json
done
grep -E "total|member|pair" $OUT/stamps_on.txt $OUT/stamps_off.txt
