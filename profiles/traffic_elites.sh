#!/bin/bash
# Where the rollout kernel's fetch above its algorithmic bytes comes from (config 2):
# FETCH_SIZE / WRITE_SIZE passes with the default 5-member elite set and with a single
# elite member (bench.py --elites 0). Per-XCD weight replication predicts
#   fetch ~= 8 XCDs x (actor + distinct elite members) + initial states,
# i.e. ~23 MB for 5 members and ~6.6 MB for one; elite switching alone would not change
# with the XCD count. Usage: bash profiles/traffic_elites.sh <tag>
set -e
TAG=${1:-te}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for el in 0,1,2,3,4 0; do
  n=$(echo $el | tr ',' '_')
  timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $OUT/fetch_e$n -o run --pmc FETCH_SIZE -- python bench.py --elites $el --steps 2 --warmup 1 --no-cpu-baseline --rollout-only --no-fit > $OUT/fetch_e$n.log 2>&1
  timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $OUT/write_e$n -o run --pmc WRITE_SIZE -- python bench.py --elites $el --steps 2 --warmup 1 --no-cpu-baseline --rollout-only --no-fit > $OUT/write_e$n.log 2>&1
  python profiles/traffic.py $OUT/fetch_e$n/run_counter_collection.csv $OUT/write_e$n/run_counter_collection.csv rollout_persist_kernel $OUT/traffic_e$n.json
done
echo done
