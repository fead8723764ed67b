#!/bin/bash
# Per-rank shard shapes (DESIGN §6 projection) + SAC MLP PMC passes, on this build.
bash profiles/gpu_shards.sh ${1:-r03sh} || exit 1
bash profiles/pmc_sac.sh gpurun_out/${1:-r03sh}/pmc_sac || exit 1
python profiles/pmc_summary.py gpurun_out/${1:-r03sh}/pmc_sac > gpurun_out/${1:-r03sh}/pmc_sac_summary.txt 2>&1
echo done
