OUT=gpurun_out/r04p
mkdir -p $OUT
export TMPDIR=/tmp
DRPO_LIB_OVERRIDE=$PWD/distributional-reachability-policy-optimization_amd/libdrpo_hip_stamps.so timeout -k 10 180 python -u profiles/sac_stamps.py > $OUT/sac_stamps.txt 2> $OUT/sac_stamps.err || exit 1
echo done
