#!/bin/bash
# Round 5: what the MLP forward's global saves cost (timing probe build with the
# epilogue saves skipped; results not used): SAC per-launch times, alternating.
OUT=gpurun_out/${1:-r05x}
mkdir -p $OUT
export TMPDIR=/tmp
LIBD=$PWD/distributional-reachability-policy-optimization_amd
for i in 1 2; do
  for t in base nosave; do
    if [ $t = base ]; then L=""; else L="DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_$t.so"; fi
    env $L timeout -k 10 180 python -u profiles/sac_micro.py --steps 10 > $OUT/sac_$t.json 2> $OUT/sac_$t.err || exit 1
    python - $OUT/sac_$t.json $t <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], ' '.join(f"{k}:{v['avg_ms']*1e3:.1f}" for k, v in d.items() if isinstance(v, dict) and 'avg_ms' in v and ':' in k))
PY
  done
done
