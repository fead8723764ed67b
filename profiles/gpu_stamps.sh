#!/bin/bash
# In-kernel phase stamps of the fused rollout kernel (profiling build libdrpo_hip_stamps.so).
set -e
OUT=gpurun_out/${1:-st}
mkdir -p $OUT
STAMPS=$PWD/distributional-reachability-policy-optimization_amd/libdrpo_hip_stamps.so
DRPO_LIB_OVERRIDE=$STAMPS DRPO_STAMPS_ROLLOUT=fused timeout -k 10 120 python profiles/stamps.py > $OUT/stamps_fused.txt 2>&1
DRPO_LIB_OVERRIDE=$STAMPS DRPO_STAMPS_ROLLOUT=fused DRPO_STAMPS_ONE_MEMBER=1 timeout -k 10 120 python profiles/stamps.py > $OUT/stamps_fused_1m.txt 2>&1
echo ok
