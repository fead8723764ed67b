set -e
mkdir -p gpurun_out/q4
S=$PWD/distributional-reachability-policy-optimization_amd/libdrpo_hip_stamps.so
DRPO_LIB_OVERRIDE=$S DRPO_STAMPS_ROLLOUT=fused timeout -k 10 120 python profiles/stamps.py > gpurun_out/q4/a.txt 2>&1
DRPO_LIB_OVERRIDE=$S DRPO_STAMPS_ROLLOUT=fused DRPO_STAMPS_ONE_MEMBER=1 timeout -k 10 120 python profiles/stamps.py > gpurun_out/q4/b.txt 2>&1
