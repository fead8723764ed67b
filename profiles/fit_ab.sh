#!/bin/bash
# Model-fit kernel A/B under rocprofv3: one kernel-trace run per variant.
# usage: bash profiles/fit_ab.sh TAG "VAR=1 OTHER=0" "VAR=0" ...   (default: split heads on / off)
set -e
TAG=${1:-ab}
shift || true
[ $# -eq 0 ] && set -- "DRPO_SPLIT_HEADS=0" "DRPO_SPLIT_HEADS=1"
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for v in "$@"; do
  echo "$v" > $OUT/v$i.env
  env $v FIT_STEPS=200 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/v$i -o fit -- python3 profiles/fit_profile.py > $OUT/v$i.log 2>&1
  i=$((i+1))
done
