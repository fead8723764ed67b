#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate runs) of the rollout kernel per bench config,
# reduced by profiles/traffic.py into gpurun_out/<tag>/traffic_rollout_fused[_cN].json
# (stamped with the library's source digest; copy them to profiles/ to attach them to
# bench lines of the same build). Usage: bash profiles/traffic_configs.sh <tag> [configs...]
set -e
TAG=${1:-t}
shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ $# -eq 0 ]; then set -- 2 3 4 5; fi
for c in "$@"; do
  timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $OUT/fetch_c$c -o run --pmc FETCH_SIZE -- python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --rollout-only --no-fit > $OUT/fetch_c$c.log 2>&1
  timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $OUT/write_c$c -o run --pmc WRITE_SIZE -- python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --rollout-only --no-fit > $OUT/write_c$c.log 2>&1
  SUF=_c$c
  if [ "$c" = "2" ]; then SUF=""; fi
  python profiles/traffic.py $OUT/fetch_c$c/run_counter_collection.csv $OUT/write_c$c/run_counter_collection.csv rollout_persist_kernel $OUT/traffic_rollout_fused$SUF.json > /dev/null
done
echo done
