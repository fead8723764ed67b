# round 4: fit phase stamps (forward split heads, paired backward with the NLL upstream)
OUT=gpurun_out/r04e
mkdir -p $OUT
export TMPDIR=/tmp
LIBD=$PWD/distributional-reachability-policy-optimization_amd
DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_stamps.so timeout -k 10 180 python -u profiles/fit_stamps.py > $OUT/fit_stamps.txt 2> $OUT/fit_stamps.err || exit 1
echo done
