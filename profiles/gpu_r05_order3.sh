#!/bin/bash
# A/B: critic forward without the actor jobs reversed (q pair, certificate, target chains;
# DRPO_SAC_CF_REVERSED, default 1) and with them (actor, q pair, certificate, qt, cc_t;
# DRPO_SAC_CFA_REVERSED).
OUT=gpurun_out/${1:-order3}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sac.py -m gpu -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  for v in R0A0 R1A0 R1A1; do
    DRPO_SAC_CF_REVERSED=${v:1:1} DRPO_SAC_CFA_REVERSED=${v:3:1} timeout -k 10 180 python -u profiles/sac_micro.py --steps 10 > $OUT/sac_micro_${v}_r$r.json 2> $OUT/sac_micro_${v}_r$r.err || exit 1
  done
  DRPO_SAC_CF_REVERSED=1 timeout -k 10 300 python -u bench.py --config 2 --steps 20 --warmup 2 --no-cpu-baseline > $OUT/bench_r$r.json 2> $OUT/bench_r$r.err || exit 1
  python -c "
import json; d=json.loads(open('$OUT/bench_r$r.json').read().strip().splitlines()[-1]); print('bench run $r sac_tf', round(d['sac']['achieved_tflops_per_gpu'],2))"
done
