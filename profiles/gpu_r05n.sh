#!/bin/bash
# Round 5: fit_fb cold vs warm body (the body run twice in one workgroup, stamps of the
# second run), and the list of translation / instruction-cache counters on this box.
OUT=gpurun_out/${1:-r05n}
mkdir -p $OUT
export TMPDIR=/tmp
LIBD=$PWD/distributional-reachability-policy-optimization_amd
DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_stamps.so timeout -k 10 120 python -u profiles/fit_stamps.py > $OUT/fit_stamps.txt 2>&1 || exit 1
DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_stamps_reps2.so timeout -k 10 120 python -u profiles/fit_stamps.py > $OUT/fit_stamps_reps2.txt 2>&1 || exit 1
grep -v "^/opt" $OUT/fit_stamps.txt | head -20; echo REPS2; grep -v "^/opt" $OUT/fit_stamps_reps2.txt | head -20
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1
grep -i -E "UTCL|TLB|ICACHE|IFETCH|INST_LEVEL|WAIT_INST" $OUT/counters.txt | head -40
