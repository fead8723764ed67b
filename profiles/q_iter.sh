#!/bin/bash
# GPU iteration: rollout + SAC parity tests, bench line, fused-rollout phase stamps.
set -e
OUT=gpurun_out/${1:-it}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_sac.py tests/test_gpu_ensemble.py tests/test_gpu_nets.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-fit > $OUT/b.json 2> $OUT/b.err
DRPO_FWD_RB=2 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-fit > $OUT/b_rb2.json 2> $OUT/b_rb2.err
STAMPS=$PWD/distributional-reachability-policy-optimization_amd/libdrpo_hip_stamps.so
DRPO_LIB_OVERRIDE=$STAMPS DRPO_STAMPS_ROLLOUT=fused timeout -k 10 120 python profiles/stamps.py > $OUT/stamps_fused.txt 2>&1
echo ok
