#!/bin/bash
# bench.py after the rollout-phase change: the 2-rank gloo bench test, default lines with
# library-event and torch-event phase bounds, config 1 (H=5) and config 5 lines.
OUT=gpurun_out/${1:-bc}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dp.py -k bench -m gpu -x -q --timeout 250 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
line() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; p=d['rollout_phase']; print('$1', round(d['value']/1e6,2), 'M/s call-bracketed', p['value_call_bracketed'] and round(p['value_call_bracketed']/1e6,2), 'frac', round(r['frac'],4), round(r['avg_launch_ms']*1e3,1), 'us', round(d['ms_per_step'],4), 'ms/step sac', round(d['sac']['value'],1), 'traffic', r.get('traffic'))"; }
timeout -k 10 200 python -u bench.py > $OUT/c2.json 2> $OUT/c2.err || exit 1
line $OUT/c2.json
DRPO_BENCH_TORCH_PHASE=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline > $OUT/c2_torch.json 2> $OUT/c2_torch.err || exit 1
line $OUT/c2_torch.json
timeout -k 10 200 python -u bench.py --no-cpu-baseline --config 1 > $OUT/c1.json 2> $OUT/c1.err || exit 1
line $OUT/c1.json
timeout -k 10 200 python -u bench.py --no-cpu-baseline --config 5 --steps 5 --warmup 2 > $OUT/c5.json 2> $OUT/c5.err || exit 1
line $OUT/c5.json
