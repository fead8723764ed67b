#!/bin/bash
# Round evidence on the current build: gpu tests, smoke, bench lines for configs
# 2-5 (config 2 with the CPU baseline) and a rocprofv3 kernel-stats pass of the
# default bench. Usage: bash profiles/gpu_final.sh <tag>
set -e
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
bash profiles/bench_configs.sh $TAG 2 3 4 5
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python bench.py --no-cpu-baseline > $OUT/stats.log 2>&1
echo done
