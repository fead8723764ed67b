#!/bin/bash
# Round 5: SAC forward phase stamps (stamps build) + layer probe with global-save variants.
OUT=gpurun_out/${1:-r05c}
mkdir -p $OUT
export TMPDIR=/tmp
LIBD=$PWD/distributional-reachability-policy-optimization_amd
DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_stamps.so timeout -k 10 180 python -u profiles/sac_fwd_stamps.py > $OUT/sac_fwd_stamps.txt 2> $OUT/sac_fwd_stamps.err || { tail $OUT/sac_fwd_stamps.err; exit 1; }
cat $OUT/sac_fwd_stamps.txt
timeout -k 10 180 ./profiles/layer_probe > $OUT/layer_probe.txt 2>&1 || exit 1
cat $OUT/layer_probe.txt
