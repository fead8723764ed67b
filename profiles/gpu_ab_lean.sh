#!/bin/bash
# GPU tests, then the bench line and the per-launch SAC timings with the lean
# 32-row forward / backward tiles on and off (DRPO_FWD_LEAN=0 DRPO_BWD_LEAN=0).
# Usage: bash profiles/gpu_ab_lean.sh <tag>
set -e
TAG=${1:-lean}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_on.json 2> $OUT/bench_on.err
DRPO_FWD_LEAN=0 DRPO_BWD_LEAN=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_off.json 2> $OUT/bench_off.err
timeout -k 10 200 python -u profiles/sac_micro.py > $OUT/micro_on.json 2> $OUT/micro_on.err
DRPO_FWD_LEAN=0 timeout -k 10 200 python -u profiles/sac_micro.py > $OUT/micro_fwdoff.json 2> $OUT/micro_fwdoff.err
DRPO_BWD_LEAN=0 timeout -k 10 200 python -u profiles/sac_micro.py > $OUT/micro_bwdoff.json 2> $OUT/micro_bwdoff.err
echo done
