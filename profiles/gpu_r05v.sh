#!/bin/bash
# Round 5: weight-gradient unit decode in 32 bits: wgrad tests, fit + SAC wgrad timings,
# setup stamps.
OUT=gpurun_out/${1:-r05v}
mkdir -p $OUT
export TMPDIR=/tmp
LIBD=$PWD/distributional-reachability-policy-optimization_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "wgrad or fit" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc $rc" >> $OUT/pytest.log; tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  FIT_STEPS=300 timeout -k 10 120 python -u profiles/fit_profile.py > $OUT/fit.log 2>&1 || exit 1
  echo "$(tail -1 $OUT/fit.log)"
  timeout -k 10 180 python -u profiles/sac_micro.py --steps 10 > $OUT/sac_micro.json 2> $OUT/sac_micro.err || exit 1
  python - $OUT/sac_micro.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(' '.join(f"{k}:{v['avg_ms']*1e3:.1f}us" for k, v in d.items() if k.startswith('mlp_wgrad') and isinstance(v, dict)))
PY
done
DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_stamps.so timeout -k 10 120 python -u profiles/wgrad_probe.py > $OUT/wgrad_probe.json 2>&1 || exit 1
python -c "
import json; d=json.loads(open('$OUT/wgrad_probe.json').read().strip().splitlines()[-1]); print(d['critic'], {k:v[:2] for k,v in d['critic_stamps'].items() if isinstance(v,list)})"
