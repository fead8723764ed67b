#!/bin/bash
# Average instruction-fetch and scalar-memory latency per kernel of the fit step
# (SQ_IFETCH_LEVEL / SQ_IFETCH, SQ_INST_LEVEL_SMEM / SQ_INSTS_SMEM).
OUT=${1:-gpurun_out/pmc_lat}
mkdir -p $OUT
export TMPDIR=/tmp
FIT_STEPS=20 timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $OUT/lat -o run \
  --pmc SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_WAVES SQ_WAVE_CYCLES \
  -- python3 profiles/fit_profile.py > $OUT/lat.log 2>&1 && \
FIT_STEPS=20 timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $OUT/ic -o run \
  --pmc SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM \
  -- python3 profiles/fit_profile.py > $OUT/ic.log 2>&1
