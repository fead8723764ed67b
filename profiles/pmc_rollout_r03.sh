#!/bin/bash
# Round-3 PMC passes of the config-2 rollout kernel (one counter group per pass, kernel
# trace only): SQ occupancy / waits / MFMA busy, L2 requests and hits, LDS.
OUT=${1:-gpurun_out/pmc_r03}
mkdir -p $OUT
export TMPDIR=/tmp
run() { timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/$1 -o run --pmc $2 -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --rollout-only > $OUT/$1.log 2>&1; }
run sq1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" || exit 1
run tcc "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" || exit 1
run lds "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" || exit 1
python profiles/pmc_summary.py $OUT rollout_persist > $OUT/summary.txt 2>&1
cat $OUT/summary.txt
