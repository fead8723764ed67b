#!/bin/bash
# Rollout-kernel variants at config 2 (existing A/B switches), rollout-only bench lines:
# default (8 waves, LDS-resident actor weights), 16 waves, no LDS-resident weights.
# Usage: bash profiles/gpu_ab_rollout.sh <tag>
set -e
OUT=gpurun_out/${1:-rab}
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --rollout-only > $OUT/base_$i.json 2> $OUT/base_$i.err
  DRPO_ROLLOUT_NW=16 timeout -k 10 200 python -u bench.py --no-cpu-baseline --rollout-only > $OUT/nw16_$i.json 2> $OUT/nw16_$i.err
  DRPO_ROLLOUT_NO_LDS_WEIGHTS=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --rollout-only > $OUT/nolw_$i.json 2> $OUT/nolw_$i.err
done
echo done
