#!/bin/bash
# Path-specialised persist kernels vs the run-time-path kernels (DRPO_ROLLOUT_PM_RUNTIME=1):
# rollout parity tests, rollout-only lines at configs 2-5 alternating.
OUT=gpurun_out/${1:-pm}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_configs.py -k rollout -m gpu -x -q --timeout 200 --timeout-method thread -rf > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
line() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$1', round(d['value']/1e6,2), 'M/s frac', round(r['frac'],4), round(r['avg_launch_ms']*1e3,1), 'us')"; }
for c in 2 3 4 5; do
  ST=20; if [ $c = 5 ]; then ST=5; fi
  for i in 1 2; do
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --rollout-only --config $c --steps $ST > $OUT/c${c}_pm_$i.json 2> $OUT/c${c}_pm_$i.err || exit 1
    line $OUT/c${c}_pm_$i.json
    DRPO_ROLLOUT_PM_RUNTIME=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --rollout-only --config $c --steps $ST > $OUT/c${c}_rt_$i.json 2> $OUT/c${c}_rt_$i.err || exit 1
    line $OUT/c${c}_rt_$i.json
  done
done
