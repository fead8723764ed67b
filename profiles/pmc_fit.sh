#!/bin/bash
# PMC passes over the model-fit micro-benchmark (profiles/fit_profile.py, config 2): one
# small counter group per pass (per-dispatch rows in the kernel-trace CSV).
OUT=${1:-gpurun_out/pmc_fit}
mkdir -p $OUT
export TMPDIR=/tmp
run() { FIT_STEPS=20 timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $OUT/$1 -o run --pmc $2 -- python3 profiles/fit_profile.py > $OUT/$1.log 2>&1; }
run ic "SQC_ICACHE_HITS SQC_ICACHE_MISSES" && \
run wv "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_BUSY_CYCLES" && \
run lds "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
