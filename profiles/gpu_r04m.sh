# minibatch prefetch A/B + GPU suite
OUT=gpurun_out/r04m
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1 || { echo pytest failed; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_pf_$i.json 2> $OUT/bench_pf_$i.err || exit 1
  DRPO_PREFETCH_BATCHES=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_nopf_$i.json 2> $OUT/bench_nopf_$i.err || exit 1
done
echo done
