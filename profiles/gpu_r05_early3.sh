#!/bin/bash
# A/B: early actor jobs first (default) vs last, and the critic forward's plain jobs
# ahead of its chain jobs (DRPO_SAC_CF_PLAIN_FIRST=1).
OUT=gpurun_out/${1:-early3}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sac.py -m gpu -q --timeout 240 --timeout-method thread -k "early or ssac_updates" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  for v in F0P0 F1P0 F1P1; do
    f=${v:1:1}; p=${v:3:1}
    DRPO_SAC_EARLY_FIRST=$f DRPO_SAC_CF_PLAIN_FIRST=$p timeout -k 10 180 python -u profiles/sac_micro.py --steps 10 > $OUT/sac_micro_${v}_r$r.json 2> $OUT/sac_micro_${v}_r$r.err || exit 1
  done
done
echo done
