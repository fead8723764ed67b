#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate runs) of the rollout kernel per bench config.
# Usage: bash profiles/traffic_configs.sh <tag> [configs...]
set -e
TAG=${1:-t}
shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ $# -eq 0 ]; then set -- 3 4 5; fi
for c in "$@"; do
  timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $OUT/fetch_c$c -o run --pmc FETCH_SIZE -- python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --rollout-only > $OUT/fetch_c$c.log 2>&1
  timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $OUT/write_c$c -o run --pmc WRITE_SIZE -- python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --rollout-only > $OUT/write_c$c.log 2>&1
done
echo done
