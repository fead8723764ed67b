#!/bin/bash
# Config-4 (tracking S=51) tile rows A/B: rollout parity tests, config-4 stamps at 32- and
# 16-row tiles (DRPO_ROLLOUT_RPT16), rollout-only bench lines alternating twice, config 2
# once (unchanged path). Usage: bash profiles/gpu_c4_ab.sh <tag>
OUT=gpurun_out/${1:-c4ab}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread -rf > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
STAMPS=$PWD/distributional-reachability-policy-optimization_amd/libdrpo_hip_stamps.so
DRPO_LIB_OVERRIDE=$STAMPS DRPO_STAMPS_CONFIG=4 DRPO_STAMPS_ROLLOUT=fused timeout -k 10 120 python profiles/stamps.py > $OUT/stamps_c4_rpt32.txt 2>&1 || exit 1
DRPO_ROLLOUT_RPT16=1 DRPO_LIB_OVERRIDE=$STAMPS DRPO_STAMPS_CONFIG=4 DRPO_STAMPS_ROLLOUT=fused timeout -k 10 120 python profiles/stamps.py > $OUT/stamps_c4_rpt16.txt 2>&1 || exit 1
line() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$1', round(d['value']/1e6,1), 'M/s frac', round(r['frac'],4), round(r['avg_launch_ms']*1e3,1), 'us')"; }
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --rollout-only --config 4 > $OUT/c4_32_$i.json 2> $OUT/c4_32_$i.err || exit 1
  line $OUT/c4_32_$i.json
  DRPO_ROLLOUT_RPT16=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --rollout-only --config 4 > $OUT/c4_16_$i.json 2> $OUT/c4_16_$i.err || exit 1
  line $OUT/c4_16_$i.json
done
timeout -k 10 200 python -u bench.py --no-cpu-baseline --rollout-only > $OUT/c2.json 2> $OUT/c2.err || exit 1
line $OUT/c2.json
cat $OUT/stamps_c4_rpt32.txt $OUT/stamps_c4_rpt16.txt
