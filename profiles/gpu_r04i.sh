# round 4: split-heads fit backward (224 workgroups) with dz + dz2 weight-gradient items
OUT=gpurun_out/r04i
mkdir -p $OUT
export TMPDIR=/tmp
LIBD=$PWD/distributional-reachability-policy-optimization_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_wgrad.py tests/test_gpu_ensemble.py tests/test_gpu_configs.py -k 'wgrad or fit or ensemble' -x -q --timeout 200 --timeout-method thread > $OUT/fit_tests.log 2>&1 || { echo fit tests failed; exit 1; }
DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_stamps.so timeout -k 10 180 python -u profiles/fit_stamps.py > $OUT/fit_stamps_split.txt 2> $OUT/fit_stamps.err || exit 1
DRPO_SPLIT_BWD=0 DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_stamps.so timeout -k 10 180 python -u profiles/fit_stamps.py > $OUT/fit_stamps_paired.txt 2>> $OUT/fit_stamps.err || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1 || { echo pytest failed; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_split_$i.json 2> $OUT/bench_split_$i.err || exit 1
  DRPO_SPLIT_BWD=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_paired_$i.json 2> $OUT/bench_paired_$i.err || exit 1
  DRPO_FIT_FUSED_ADAM=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_sepadam_$i.json 2> $OUT/bench_sepadam_$i.err || exit 1
done
echo done
