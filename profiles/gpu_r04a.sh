OUT=gpurun_out/r04a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u profiles/host_probe.py > $OUT/host_probe.json 2> $OUT/host_probe.err || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python bench.py --no-cpu-baseline --no-fit > $OUT/stats.log 2>&1 || exit 1
echo done
