# fit 200x200 layers balanced over the SIMDs (tile_dense_13s): tests, stamps, bench A/B
OUT=gpurun_out/r04n
mkdir -p $OUT
export TMPDIR=/tmp
LIBD=$PWD/distributional-reachability-policy-optimization_amd
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1 || { echo pytest failed; exit 1; }
DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_stamps.so timeout -k 10 180 python -u profiles/fit_stamps.py > $OUT/fit_stamps.txt 2> $OUT/stamps.err || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_13s_$i.json 2> $OUT/bench_13s_$i.err || exit 1
  DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_n13.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_n13_$i.json 2> $OUT/bench_n13_$i.err || exit 1
done
echo done
