# round 4: forward row-block A/B (16- vs 32-row tiles in the SAC multi-job forward),
# SAC PMC passes, rocprofv3 stats of the default bench
OUT=gpurun_out/r04h
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_rb1_$i.json 2> $OUT/bench_rb1_$i.err || exit 1
  DRPO_FWD_RB=2 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_rb2_$i.json 2> $OUT/bench_rb2_$i.err || exit 1
done
bash profiles/pmc_sac.sh $OUT/pmc_sac || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python bench.py --no-cpu-baseline > $OUT/stats.log 2>&1 || exit 1
echo done
