#!/bin/bash
# A/B: the actor update's first forward inside the critic update's forward launch
# (DRPO_SAC_EARLY_ACTOR=1, default) vs its own 'a.f1' launch (=0).
OUT=gpurun_out/${1:-early}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sac.py -m gpu -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  for v in 0 1; do
    DRPO_SAC_EARLY_ACTOR=$v timeout -k 10 180 python -u profiles/sac_micro.py --steps 10 > $OUT/sac_micro_e${v}_r$r.json 2> $OUT/sac_micro_e${v}_r$r.err || exit 1
    DRPO_SAC_EARLY_ACTOR=$v timeout -k 10 300 python -u bench.py --config 2 --steps 20 --warmup 2 --no-cpu-baseline > $OUT/bench_e${v}_r$r.json 2> $OUT/bench_e${v}_r$r.err || exit 1
    python -c "
import json; d=json.loads(open('$OUT/bench_e${v}_r$r.json').read().strip().splitlines()[-1]); s=d['sac']
print('early=$v run=$r', 'sac_tf', round(s['achieved_tflops_per_gpu'],2), {k: s[k] for k in s if 'ms' in k})"
  done
done
