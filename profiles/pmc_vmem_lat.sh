#!/bin/bash
# Average vector-memory latency of the rollout kernel (and the SAC kernels):
# SQ_INST_LEVEL_VMEM / SQ_INSTS_VMEM_RD (+ LDS), one counter group per run.
# Usage: bash profiles/pmc_vmem_lat.sh <tag>
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $OUT/lat -o run \
  --pmc SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM \
  -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fit > $OUT/lat.log 2>&1 || exit 1
python3 profiles/pmc_summary.py $OUT > $OUT/summary.txt 2>&1
python3 - $OUT/summary.txt << 'PY'
import re, sys
cur, d = None, {}
for line in open(sys.argv[1]):
    if not line.startswith(' '):
        cur = line.strip(); d[cur] = {}
    else:
        p = line.split()
        d[cur][p[0]] = float(p[1])
for k, c in d.items():
    if c.get('SQ_INSTS_VMEM_RD'):
        print(f"{k[:60]:60s} vmem lat {c['SQ_INST_LEVEL_VMEM'] / c['SQ_INSTS_VMEM_RD']:8.1f}  lds lat {c.get('SQ_INST_LEVEL_LDS', 0) / max(1, c.get('SQ_INSTS_LDS', 1)):7.1f}")
PY
