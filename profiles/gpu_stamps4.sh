#!/bin/bash
# config-4 stamps: elites as configured vs one member (L2-warm member weights)
OUT=gpurun_out/${1:-st4}
mkdir -p $OUT
STAMPS=$PWD/distributional-reachability-policy-optimization_amd/libdrpo_hip_stamps.so
DRPO_STAMPS_CONFIG=4 DRPO_LIB_OVERRIDE=$STAMPS DRPO_STAMPS_ROLLOUT=fused timeout -k 10 120 python profiles/stamps.py > $OUT/stamps_c4.txt 2>&1 || exit 1
DRPO_STAMPS_ONE_MEMBER=1 DRPO_STAMPS_CONFIG=4 DRPO_LIB_OVERRIDE=$STAMPS DRPO_STAMPS_ROLLOUT=fused timeout -k 10 120 python profiles/stamps.py > $OUT/stamps_c4_1m.txt 2>&1 || exit 1
echo done
