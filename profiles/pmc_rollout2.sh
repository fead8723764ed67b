#!/bin/bash
# Counter list of the box + SQ / TA / TCP passes over the rollout-only bench (config 2).
# One counter group per pass, kernel trace only. Usage: bash profiles/pmc_rollout2.sh <outdir>
OUT=${1:-gpurun_out/pmc2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > $OUT/list_avail.txt 2>&1 || true
run() { timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/$1 -o run --pmc $2 -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --rollout-only > $OUT/$1.log 2>&1; }
run sq1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" || exit 1
run sq2 "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MFMA SQ_INST_CYCLES_VMEM" || exit 1
echo done
