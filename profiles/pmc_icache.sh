#!/bin/bash
# Instruction-fetch counters of the rollout kernel (bench --rollout-only) and of the SAC
# update's kernels (sac_micro): instruction-cache requests / misses and the average
# instruction-fetch latency (SQ_IFETCH_LEVEL / SQ_IFETCH). One counter group per run.
# Usage: bash profiles/pmc_icache.sh <tag>
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
run() {   # name, counters, command...
  local n=$1 c=$2; shift 2
  timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $OUT/$n -o run --pmc $c -- "$@" > $OUT/$n.log 2>&1
}
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fit"
run ic_b "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" $B || exit 1
run if_b "SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" $B || exit 1
python3 profiles/pmc_summary.py $OUT > $OUT/summary.txt 2>&1
cat $OUT/summary.txt | head -60
