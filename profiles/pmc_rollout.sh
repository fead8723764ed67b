#!/bin/bash
# PMC passes for the rollout step kernel (one counter group per pass; never combined
# with trace domains). Usage on the GPU box: bash profiles/pmc_rollout.sh <outdir>
set -e
OUT=${1:-gpurun_out/pmc}
mkdir -p $OUT
export TMPDIR=/tmp
run() { timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/$1 -o run --pmc $2 -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline --rollout-only > $OUT/$1.log 2>&1; }
run sq1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES"
run fetch "FETCH_SIZE"
run write "WRITE_SIZE"
run tcc "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum"
run lds "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
