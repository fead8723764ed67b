#!/bin/bash
# Per-rank shard shapes of the multi-GPU configs, measured on ONE GPU (DESIGN §6
# projection; the 8-GPU RCCL run itself is the driver's):
#   config 5 on 8 ranks: each rank rolls out / updates B = 65536 / 8 = 8192 rows and fits
#     E / 8 = 4 members (MemberShard);
#   config 4 on 4 ranks: each rank fits E / 4 = 2 members (and rolls out its own B = 16384).
# Usage: bash profiles/gpu_shards.sh <tag>
OUT=gpurun_out/${1:-shards}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 5 --global-batch 8192 --steps 5 --warmup 2 > $OUT/c5_rank_b8192.json 2> $OUT/c5_rank_b8192.err || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 5 --global-batch 8192 --ensemble 4 --steps 3 --warmup 1 > $OUT/c5_rank_e4.json 2> $OUT/c5_rank_e4.err || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 4 --ensemble 2 --steps 3 --warmup 1 > $OUT/c4_rank_e2.json 2> $OUT/c4_rank_e2.err || exit 1
echo done
