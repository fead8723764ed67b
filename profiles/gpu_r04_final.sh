#!/bin/bash
# Round-4 evidence on the final build: GPU suite, smoke, bench lines for configs 1-5
# (config 2 with the CPU baseline), rocprofv3 kernel stats of the default bench, and the
# FETCH / WRITE passes of the rollout kernel per config (digest-stamped traffic JSONs).
# Usage: bash profiles/gpu_r04_final.sh <tag>
OUT=gpurun_out/${1:-r04final}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1
echo "pytest rc $?" >> $OUT/pytest_gpu.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
bash profiles/bench_configs.sh ${1:-r04final} 1 2 3 4 5 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python bench.py --no-cpu-baseline > $OUT/stats.log 2>&1 || exit 1
bash profiles/traffic_configs.sh ${1:-r04final} 2 3 4 5 || exit 1
echo done
