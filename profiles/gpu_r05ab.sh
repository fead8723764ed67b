#!/bin/bash
# Round 5: the multiplier forward as a post chain of the constraint-bound job
# (DRPO_SAC_POST_MULT): SAC parity tests, then SAC per-update A/B, three rounds.
OUT=gpurun_out/${1:-r05ab}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_sac.py tests/test_gpu_configs.py tests/test_gpu_trainer.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -rf > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc $rc" >> $OUT/pytest.log; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit 1
for i in 1 2 3; do
  for v in 1 0; do
    DRPO_SAC_POST_MULT=$v timeout -k 10 180 python -u profiles/sac_micro.py --steps 10 > $OUT/sac_$v_$i.json 2> $OUT/sac.err || exit 1
    python - $OUT/sac_$v_$i.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
tot = sum(v['ms'] for k, v in d.items() if isinstance(v, dict) and 'ms' in v and ':' not in k)
print('post', sys.argv[2], f"all-kernels {tot:.2f} ms", ' '.join(f"{k}:{v['avg_ms']*1e3:.1f}" for k, v in d.items() if isinstance(v, dict) and 'avg_ms' in v and (k.startswith('mlp_fwd:a') or k.startswith('mlp_fwd:m'))))
PY
  done
done
