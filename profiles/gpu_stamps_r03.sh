#!/bin/bash
# Per-phase stamps of the final build's persist kernel at configs 2, 3 and 4.
OUT=gpurun_out/${1:-st3}
mkdir -p $OUT
STAMPS=$PWD/distributional-reachability-policy-optimization_amd/libdrpo_hip_stamps.so
for c in 2 3 4; do
  DRPO_LIB_OVERRIDE=$STAMPS DRPO_STAMPS_CONFIG=$c DRPO_STAMPS_ROLLOUT=fused timeout -k 10 120 python profiles/stamps.py > $OUT/stamps_c$c.txt 2>&1 || exit 1
done
cat $OUT/stamps_c2.txt $OUT/stamps_c3.txt
