#!/bin/bash
# Default order (actor, plain, chains with the early actor jobs; chains, plain without)
# against the previous default (chains, plain, actor): per-launch times and SAC TFLOP/s.
OUT=gpurun_out/${1:-early4}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sac.py -m gpu -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export DRPO_SAC_EARLY_FIRST=0 DRPO_SAC_CF_PLAIN_FIRST=0; else unset DRPO_SAC_EARLY_FIRST DRPO_SAC_CF_PLAIN_FIRST; fi
    timeout -k 10 180 python -u profiles/sac_micro.py --steps 10 > $OUT/sac_micro_${v}_r$r.json 2> $OUT/sac_micro_${v}_r$r.err || exit 1
    timeout -k 10 300 python -u bench.py --config 2 --steps 20 --warmup 2 --no-cpu-baseline > $OUT/bench_${v}_r$r.json 2> $OUT/bench_${v}_r$r.err || exit 1
    python -c "
import json; d=json.loads(open('$OUT/bench_${v}_r$r.json').read().strip().splitlines()[-1]); s=d['sac']
print('$v run=$r', 'sac_tf', round(s['achieved_tflops_per_gpu'],2))"
  done
done
