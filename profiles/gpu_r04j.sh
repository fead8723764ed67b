# round 4: fit split backward + fused Adam (tests, stamps, bench A/B) and the SIMD-balanced
# rollout member layer (tests, stamps, bench A/B)
OUT=gpurun_out/r04j
mkdir -p $OUT
export TMPDIR=/tmp
LIBD=$PWD/distributional-reachability-policy-optimization_amd
timeout -k 10 500 python -u -m pytest tests/test_gpu_wgrad.py tests/test_gpu_ensemble.py tests/test_gpu_rollout.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $OUT/tests_a.log 2>&1 || { echo tests failed; exit 1; }
DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_stamps.so timeout -k 10 180 python -u profiles/fit_stamps.py > $OUT/fit_stamps_split.txt 2> $OUT/stamps.err || exit 1
DRPO_SPLIT_BWD=0 DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_stamps.so timeout -k 10 180 python -u profiles/fit_stamps.py > $OUT/fit_stamps_paired.txt 2>> $OUT/stamps.err || exit 1
DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_stamps.so timeout -k 10 180 python -u profiles/stamps.py > $OUT/stamps_m2split.txt 2>> $OUT/stamps.err || exit 1
DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_stamps_m2off.so timeout -k 10 180 python -u profiles/stamps.py > $OUT/stamps_m2off.txt 2>> $OUT/stamps.err || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1 || { echo pytest failed; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_new_$i.json 2> $OUT/bench_new_$i.err || exit 1
  DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_m2off.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_m2off_$i.json 2> $OUT/bench_m2off_$i.err || exit 1
  DRPO_SPLIT_BWD=0 DRPO_FIT_FUSED_ADAM=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_oldfit_$i.json 2> $OUT/bench_oldfit_$i.err || exit 1
done
echo done
