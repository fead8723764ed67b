#!/bin/bash
# Instruction-cache PMC passes over the rollout-only bench (one small group per pass).
set -e
OUT=${1:-gpurun_out/ic}
mkdir -p $OUT
export TMPDIR=/tmp
run() { timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $OUT/$1 -o run --pmc $2 -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-fit $3 > $OUT/$1.log 2>&1; }
run ic "SQC_ICACHE_HITS SQC_ICACHE_MISSES" --rollout-only
run wi "SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_IFETCH" --rollout-only
run icsac "SQC_ICACHE_HITS SQC_ICACHE_MISSES" ""
