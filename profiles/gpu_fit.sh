#!/bin/bash
# model-fit kernels (rocprofv3 stats) + the default bench line
OUT=gpurun_out/${1:-fit}
mkdir -p $OUT
export TMPDIR=/tmp
FIT_STEPS=200 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/fit -o fit -- python3 profiles/fit_profile.py > $OUT/fit.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 > $OUT/bench.json 2> $OUT/bench.err || exit 1
echo done
