#!/bin/bash
# Round-3 re-entry pass: GPU suite, smoke, config-2 bench line (with CPU baseline),
# rocprofv3 kernel stats of the default bench, fused-rollout phase stamps.
OUT=gpurun_out/${1:-r03s}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=30 --timeout 300 --timeout-method thread -rf > $OUT/pytest.log 2>&1
echo "pytest rc $?" >> $OUT/pytest.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python bench.py --no-cpu-baseline > $OUT/stats.log 2>&1 || exit 1
bash profiles/gpu_stamps.sh ${1:-r03s} || exit 1
echo done
