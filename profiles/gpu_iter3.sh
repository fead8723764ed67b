#!/bin/bash
# quick rollout iteration: rollout parity tests, A/B bench lines at config 2 (v2 vs v1),
# fused-kernel stamps, config-3/4 rollout-only lines. Usage: bash profiles/gpu_iter3.sh <tag>
OUT=gpurun_out/${1:-it}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_rollout.py tests/test_gpu_noise.py -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread -rf > $OUT/pytest.log 2>&1
echo "pytest rc $?" >> $OUT/pytest.log
for i in 1 2; do
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-fit --rollout-only --steps 10 > $OUT/bench_v2_$i.json 2> $OUT/bench_v2_$i.err || exit 1
DRPO_ROLLOUT_V1=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-fit --rollout-only --steps 10 > $OUT/bench_v1_$i.json 2> $OUT/bench_v1_$i.err || exit 1
done
STAMPS=$PWD/distributional-reachability-policy-optimization_amd/libdrpo_hip_stamps.so
DRPO_LIB_OVERRIDE=$STAMPS DRPO_STAMPS_ROLLOUT=fused timeout -k 10 120 python profiles/stamps.py > $OUT/stamps_fused.txt 2>&1 || exit 1
for c in 3 4; do
timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-fit --rollout-only --steps 5 > $OUT/bench_c$c.json 2> $OUT/bench_c$c.err || exit 1
DRPO_ROLLOUT_V1=1 timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-fit --rollout-only --steps 5 > $OUT/bench_c${c}_v1.json 2> $OUT/bench_c${c}_v1.err || exit 1
done
echo done
