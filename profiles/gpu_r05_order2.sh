#!/bin/bash
# A/B: reversed item order of the critic weight-gradient launch, reversed critic forward.
OUT=gpurun_out/${1:-order2}
mkdir -p $OUT
export TMPDIR=/tmp
DRPO_SAC_REVERSE=c.wg timeout -k 10 300 python -u -m pytest tests/test_gpu_sac.py -m gpu -q --timeout 240 --timeout-method thread -k "ssac_updates" > $OUT/pytest_rev.log 2>&1 || { tail -30 $OUT/pytest_rev.log; exit 1; }
tail -1 $OUT/pytest_rev.log
for r in 1 2; do
  for v in none c.wg c.f; do
    DRPO_SAC_REVERSE=$v timeout -k 10 180 python -u profiles/sac_micro.py --steps 10 > $OUT/sac_micro_${v}_r$r.json 2> $OUT/sac_micro_${v}_r$r.err || exit 1
  done
done
echo done
