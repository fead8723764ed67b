set -e
mkdir -p gpurun_out/q5
S=$PWD/distributional-reachability-policy-optimization_amd/libdrpo_hip_stamps.so
DRPO_LIB_OVERRIDE=$S DRPO_STAMPS_ROLLOUT=fused DRPO_STAMPS_HM=256 timeout -k 10 120 python profiles/stamps.py > gpurun_out/q5/a.txt 2>&1
DRPO_LIB_OVERRIDE=$S DRPO_STAMPS_ROLLOUT=fused DRPO_STAMPS_HM=192 timeout -k 10 120 python profiles/stamps.py > gpurun_out/q5/b.txt 2>&1
