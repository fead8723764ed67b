#!/bin/bash
# Round-6 evidence, part B: bench lines for configs 1-5 (config 2 with the CPU baseline;
# traffic attached from the digest-stamped JSONs in profiles/) and the default line.
OUT=gpurun_out/${1:-r06final}
mkdir -p $OUT
export TMPDIR=/tmp
bash profiles/bench_configs.sh ${1:-r06final} 1 2 3 4 5 || exit 1
timeout -k 10 400 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
python profiles/summ.py $OUT/bench_c*.json $OUT/bench_default.json
