#!/bin/bash
# PMC passes over the SAC update micro-run (profiles/sac_micro.py): one counter group
# per pass, kernel-trace only (never with sys/runtime trace domains).
# Usage on the GPU box: bash profiles/pmc_sac.sh <outdir>
set -e
OUT=${1:-gpurun_out/pmc_sac}
mkdir -p $OUT
export TMPDIR=/tmp
run() { timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/$1 -o run --pmc $2 -- python profiles/sac_micro.py --steps 2 > $OUT/$1.log 2>&1; }
run sq1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES"
run lds "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
run tcc "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum"
run fetch "FETCH_SIZE"
