#!/bin/bash
# Quick GPU iteration: gpu tests, bench line, fused-rollout and MLP phase stamps.
set -e
OUT=gpurun_out/${1:-q}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
STAMPS=$PWD/distributional-reachability-policy-optimization_amd/libdrpo_hip_stamps.so
if [ -f $STAMPS ]; then
DRPO_LIB_OVERRIDE=$STAMPS DRPO_STAMPS_ROLLOUT=fused timeout -k 10 120 python profiles/stamps.py > $OUT/stamps_fused.txt 2>&1
DRPO_LIB_OVERRIDE=$STAMPS timeout -k 10 120 python profiles/stamps.py > $OUT/stamps_mlp.txt 2>&1
fi
echo done
