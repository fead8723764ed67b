#!/bin/bash
# rollout stamps (phase F detail) + model-fit kernels + ensemble / SAC parity tests
OUT=gpurun_out/${1:-it4}
mkdir -p $OUT
export TMPDIR=/tmp
STAMPS=$PWD/distributional-reachability-policy-optimization_amd/libdrpo_hip_stamps.so
DRPO_LIB_OVERRIDE=$STAMPS DRPO_STAMPS_ROLLOUT=fused timeout -k 10 120 python profiles/stamps.py > $OUT/stamps_fused.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_ensemble.py tests/test_gpu_sac.py tests/test_gpu_fullwidth.py tests/test_gpu_configs.py -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread -rf > $OUT/pytest.log 2>&1
echo "pytest rc $?" >> $OUT/pytest.log
FIT_STEPS=200 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/fit -o fit -- python3 profiles/fit_profile.py > $OUT/fit.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 > $OUT/bench.json 2> $OUT/bench.err || exit 1
echo done
