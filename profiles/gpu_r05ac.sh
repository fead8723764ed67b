#!/bin/bash
# Round 5: multi-job forward with the slots interleaved along grid x (DRPO_FWD_INTERLEAVE):
# SAC per-update A/B, three alternating rounds.
OUT=gpurun_out/${1:-r05ac}
mkdir -p $OUT
export TMPDIR=/tmp
LIBD=$PWD/distributional-reachability-policy-optimization_amd
for i in 1 2 3; do
  for t in base ilv; do
    if [ $t = base ]; then L=""; else L="DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_$t.so"; fi
    env $L timeout -k 10 180 python -u profiles/sac_micro.py --steps 10 > $OUT/sac_${t}_$i.json 2> $OUT/sac.err || exit 1
    python - $OUT/sac_${t}_$i.json $t <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
tot = sum(v['ms'] for k, v in d.items() if isinstance(v, dict) and 'ms' in v and ':' not in k)
print(sys.argv[2], f"all-kernels {tot:.2f} ms", ' '.join(f"{k}:{v['avg_ms']*1e3:.1f}" for k, v in d.items() if isinstance(v, dict) and 'avg_ms' in v and k.startswith('mlp_fwd:')))
PY
  done
done
