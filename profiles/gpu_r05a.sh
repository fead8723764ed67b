#!/bin/bash
# Round-5 baseline: per-launch SAC timings (no profiler), fit micro-benchmark, default bench,
# rocprofv3 kernel stats of the SAC micro-run.
OUT=gpurun_out/${1:-r05a}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 180 python -u profiles/sac_micro.py --steps 10 > $OUT/sac_micro.json 2> $OUT/sac_micro.err || exit 1
timeout -k 10 180 python -u profiles/fit_profile.py > $OUT/fit.txt 2> $OUT/fit.err || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python profiles/sac_micro.py --steps 5 > $OUT/stats.log 2>&1 || exit 1
echo done
