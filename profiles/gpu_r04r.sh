OUT=gpurun_out/${1:-r04r}
mkdir -p $OUT
export TMPDIR=/tmp
LIBD=$PWD/distributional-reachability-policy-optimization_amd
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1
echo "pytest rc $?" >> $OUT/pytest_gpu.log
DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_stamps.so timeout -k 10 180 python -u profiles/sac_stamps.py > $OUT/sac_stamps.txt 2> $OUT/stamps.err || exit 1
for i in 1 2; do timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_$i.json 2> $OUT/bench_$i.err || exit 1; done
echo done
