#!/bin/bash
# A/B: position of the early actor jobs in the critic forward launch (last vs first).
OUT=gpurun_out/${1:-early2}
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for v in 0 1; do
    DRPO_SAC_EARLY_FIRST=$v timeout -k 10 180 python -u profiles/sac_micro.py --steps 10 > $OUT/sac_micro_f${v}_r$r.json 2> $OUT/sac_micro_f${v}_r$r.err || exit 1
  done
done
echo done
