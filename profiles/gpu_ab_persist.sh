#!/bin/bash
# A/B of the persistent rollout kernel's build knobs (csrc/rollout.hip: DRPO_PERSIST_KARG,
# DRPO_PREFETCH_M1, DRPO_ABIAS_LDS), each built by build_lib.py --tag <v>:
#   per variant: config-2 per-phase stamps, and rollout-only bench lines at configs 2, 3
#   and 4 (two alternating rounds at config 2).
# Usage: bash profiles/gpu_ab_persist.sh <outdir-tag> <variant>...   (variant "base" = default build)
OUT=gpurun_out/${1:-abp}
shift
mkdir -p $OUT
export TMPDIR=/tmp
D=$PWD/distributional-reachability-policy-optimization_amd
lib() { if [ "$1" = base ]; then echo $D/libdrpo_hip$2.so; else echo $D/libdrpo_hip$2_$1.so; fi; }
for v in "$@"; do
  DRPO_LIB_OVERRIDE=$(lib $v _stamps) DRPO_STAMPS_CONFIG=2 DRPO_STAMPS_ROLLOUT=fused timeout -k 10 120 python profiles/stamps.py > $OUT/stamps_$v.txt 2>&1 || exit 1
done
for i in 1 2; do
  for v in "$@"; do
    DRPO_LIB_OVERRIDE=$(lib $v) timeout -k 10 200 python -u bench.py --no-cpu-baseline --rollout-only > $OUT/c2_${v}_$i.json 2> $OUT/c2_${v}_$i.err || exit 1
  done
done
for c in 3 4; do
  for v in "$@"; do
    DRPO_LIB_OVERRIDE=$(lib $v) timeout -k 10 200 python -u bench.py --no-cpu-baseline --rollout-only --config $c > $OUT/c${c}_${v}.json 2> $OUT/c${c}_${v}.err || exit 1
  done
done
echo done
