#!/bin/bash
# rollout iteration: parity tests, bench lines at configs 2-4 (rollout only), stamps at configs 2 and 4
OUT=gpurun_out/${1:-it5}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_rollout.py tests/test_gpu_noise.py -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread -rf > $OUT/pytest.log 2>&1
echo "pytest rc $?" >> $OUT/pytest.log
for c in 2 3 4; do
timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-fit --rollout-only --steps 10 > $OUT/bench_c$c.json 2> $OUT/bench_c$c.err || exit 1
done
STAMPS=$PWD/distributional-reachability-policy-optimization_amd/libdrpo_hip_stamps.so
for c in 2 4; do
DRPO_STAMPS_CONFIG=$c DRPO_LIB_OVERRIDE=$STAMPS DRPO_STAMPS_ROLLOUT=fused timeout -k 10 120 python profiles/stamps.py > $OUT/stamps_c$c.txt 2>&1 || exit 1
done
echo done
