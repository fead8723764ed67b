#!/bin/bash
# stamps only (profiling build)
OUT=gpurun_out/${1:-st}
mkdir -p $OUT
STAMPS=$PWD/distributional-reachability-policy-optimization_amd/libdrpo_hip_stamps.so
DRPO_LIB_OVERRIDE=$STAMPS DRPO_STAMPS_ROLLOUT=fused timeout -k 10 120 python profiles/stamps.py > $OUT/stamps_fused.txt 2>&1
echo done
