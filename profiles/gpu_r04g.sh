# round 4: kernel floor probe; warm-up touches A/B (fit stamps + bench), GPU tests
OUT=gpurun_out/r04g
mkdir -p $OUT
export TMPDIR=/tmp
LIBD=$PWD/distributional-reachability-policy-optimization_amd
timeout -k 10 60 ./profiles/karg_probe > $OUT/karg_probe.txt 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kstats -o run -- ./profiles/karg_probe > $OUT/karg_prof.log 2>&1 || exit 1
for v in stamps stamps_nt; do DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_$v.so timeout -k 10 180 python -u profiles/fit_stamps.py > $OUT/fit_$v.txt 2> $OUT/fit_$v.err || exit 1; done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1 || { echo pytest failed; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_t$i.json 2> $OUT/bench_t$i.err || exit 1
  DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_nt.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_nt$i.json 2> $OUT/bench_nt$i.err || exit 1
done
echo done
