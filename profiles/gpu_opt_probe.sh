#!/bin/bash
# Optimizer timing probe (DRPO_OPT_PROBE: 1 = no transposed-mirror stores, 2 = no mirror
# stores; results invalid, timing only): config-2 bench lines, fit ms and SAC TFLOP/s,
# plus rocprofv3 kernel stats of the fit micro-run per probe value.
OUT=gpurun_out/${1:-optp}
mkdir -p $OUT
export TMPDIR=/tmp
line() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); s=d['sac']
print('$1', 'sac', round(s['achieved_tflops_per_gpu'],1), 'TF fit', round(d['model_fit']['ms_per_fit_step'],4), 'ms')"; }
for i in 1 2; do
  for p in 0 1 2; do
    DRPO_OPT_PROBE=$p timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 5 > $OUT/p${p}_$i.json 2> $OUT/p${p}_$i.err || exit 1
    line $OUT/p${p}_$i.json
  done
done
for p in 0 1 2; do
  DRPO_OPT_PROBE=$p timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/st$p -o run -- python profiles/fit_profile.py > $OUT/st$p.log 2>&1 || exit 1
  grep -h "optim_step" $OUT/st$p/run_kernel_stats.csv | cut -d, -f1-4
done
