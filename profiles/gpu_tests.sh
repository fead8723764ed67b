#!/bin/bash
# GPU test pass: the given pytest arguments (default: tests), one pytest process,
# per-test timeout; log under gpurun_out/<tag>/. Usage: bash profiles/gpu_tests.sh <tag> [pytest args...]
set -e
TAG=${1:-t}
shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ $# -eq 0 ]; then set -- tests; fi
timeout -k 10 1000 python -u -m pytest "$@" -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
echo done
