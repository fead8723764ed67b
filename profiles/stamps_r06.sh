#!/bin/bash
# Stamps build (libdrpo_hip_stamps.so): rollout phases + core sub-phases at config 2 and
# 3, the SAC multi-job forward phases, the fit kernel phases. Usage: bash profiles/stamps_r06.sh <tag>
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
ST=$PWD/distributional-reachability-policy-optimization_amd/libdrpo_hip_stamps.so
for c in 2 3; do
  DRPO_STAMPS_H=3 DRPO_STAMPS_CONFIG=$c DRPO_LIB_OVERRIDE=$ST DRPO_STAMPS_ROLLOUT=fused timeout -k 10 120 python profiles/stamps.py > $OUT/stamps_c$c.txt 2>&1 || exit 1
done
DRPO_LIB_OVERRIDE=$ST timeout -k 10 120 python -u profiles/sac_fwd_stamps.py > $OUT/sac_fwd_stamps.txt 2>&1 || exit 1
DRPO_LIB_OVERRIDE=$ST timeout -k 10 120 python -u profiles/fit_stamps.py > $OUT/fit_stamps.txt 2>&1 || exit 1
cat $OUT/stamps_c2.txt $OUT/stamps_c3.txt
