#!/bin/bash
# v2 rollout kernel: GPU suite, A/B bench lines (v2 vs v1 structure) at config 2, stamps,
# bench lines at configs 3-5.
OUT=gpurun_out/r03c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --maxfail=30 --timeout 400 --timeout-method thread -rf > $OUT/pytest.log 2>&1
echo "pytest rc $?" >> $OUT/pytest.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-fit --steps 10 > $OUT/bench_v2_$i.json 2> $OUT/bench_v2_$i.err || exit 1
DRPO_ROLLOUT_V1=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-fit --steps 10 > $OUT/bench_v1_$i.json 2> $OUT/bench_v1_$i.err || exit 1
done
STAMPS=$PWD/distributional-reachability-policy-optimization_amd/libdrpo_hip_stamps.so
DRPO_LIB_OVERRIDE=$STAMPS DRPO_STAMPS_ROLLOUT=fused timeout -k 10 120 python profiles/stamps.py > $OUT/stamps_fused.txt 2>&1 || exit 1
for c in 3 4 5; do
timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-fit --steps 5 > $OUT/bench_c$c.json 2> $OUT/bench_c$c.err || exit 1
done
echo done
