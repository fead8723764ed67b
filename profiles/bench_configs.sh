#!/bin/bash
# Bench line per BASELINE config (1-GPU), default config 2 with the CPU baseline.
# Usage: bash profiles/bench_configs.sh <tag> [configs...]
set -e
TAG=${1:-b}
shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ $# -eq 0 ]; then set -- 1 2 3 4 5; fi
for c in "$@"; do
  EXTRA="--no-cpu-baseline"
  if [ "$c" = "2" ]; then EXTRA=""; fi
  STEPS=20
  if [ "$c" = "5" ]; then STEPS=5; fi
  timeout -k 10 400 python -u bench.py --config $c --steps $STEPS --warmup 2 $EXTRA > $OUT/bench_c$c.json 2> $OUT/bench_c$c.err
done
echo done
