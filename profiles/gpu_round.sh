#!/bin/bash
# One GPU-box pass: gpu tests, smoke, the default bench line, a rocprofv3 kernel
# stats pass of the same bench command, and FETCH/WRITE PMC passes (separate runs)
# for the rollout kernel's HBM traffic. Usage: bash profiles/gpu_round.sh <tag>
set -e
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python bench.py --no-cpu-baseline > $OUT/stats.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/fetch -o run --pmc FETCH_SIZE -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline --rollout-only > $OUT/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/write -o run --pmc WRITE_SIZE -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline --rollout-only > $OUT/write.log 2>&1
echo done
