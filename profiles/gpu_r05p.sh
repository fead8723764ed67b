#!/bin/bash
# Round 5: early finish loads + transposed refresh through LDS: GPU suite, fit
# and SAC A/B (DRPO_WGRAD_VF=0 / 1), stamps.
OUT=gpurun_out/${1:-r05p}
mkdir -p $OUT
export TMPDIR=/tmp
LIBD=$PWD/distributional-reachability-policy-optimization_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_wgrad.py tests/test_gpu_sac.py -m gpu -x -q --timeout 300 --timeout-method thread -rf > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc $rc" >> $OUT/pytest.log; tail -4 $OUT/pytest.log
[ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for v in "X=1" "DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_noptt.so" "DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_noearly.so"; do
    env $v FIT_STEPS=300 timeout -k 10 120 python -u profiles/fit_profile.py > $OUT/fit.log 2>&1 || exit 1
    echo "[$v]: $(tail -1 $OUT/fit.log)"
    env $v timeout -k 10 180 python -u profiles/sac_micro.py --steps 10 > $OUT/sac_micro.json 2> $OUT/sac_micro.err || exit 1
    python - $OUT/sac_micro.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(' '.join(f"{k}:{v['avg_ms']*1e3:.1f}us" for k, v in d.items() if k.startswith('mlp_wgrad') and isinstance(v, dict)))
PY
  done
done
DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_stamps.so timeout -k 10 120 python -u profiles/fit_stamps.py > $OUT/fit_stamps.txt 2>&1 || exit 1
grep -v "^/opt" $OUT/fit_stamps.txt | tail -7
