#!/bin/bash
# Round-6 evidence on the final build, part A: GPU suite, smoke, the rollout kernel's
# FETCH / WRITE passes per config (digest-stamped traffic JSONs), rocprofv3 kernel stats
# of the default bench, rollout stamps (configs 2-4), fit stamps, SAC micro-run.
# Part B (after the traffic JSONs are copied into profiles/): bench_configs.sh + default.
# Usage: bash profiles/gpu_r06_final.sh <tag>
OUT=gpurun_out/${1:-r06final}
mkdir -p $OUT
export TMPDIR=/tmp
STAMPS=$PWD/distributional-reachability-policy-optimization_amd/libdrpo_hip_stamps.so
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc $rc" >> $OUT/pytest_gpu.log; tail -2 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
tail -1 $OUT/smoke.log
bash profiles/traffic_configs.sh ${1:-r06final} 2 3 4 5 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python bench.py --no-cpu-baseline > $OUT/stats.log 2>&1 || exit 1
for c in 2 3 4; do
  DRPO_STAMPS_H=3 DRPO_STAMPS_CONFIG=$c DRPO_LIB_OVERRIDE=$STAMPS DRPO_STAMPS_ROLLOUT=fused timeout -k 10 120 python profiles/stamps.py > $OUT/stamps_c$c.txt 2>&1 || exit 1
done
DRPO_LIB_OVERRIDE=$STAMPS timeout -k 10 120 python -u profiles/fit_stamps.py > $OUT/fit_stamps.txt 2>&1 || exit 1
timeout -k 10 180 python -u profiles/sac_micro.py --steps 10 > $OUT/sac_micro.json 2> $OUT/sac_micro.err || exit 1
grep total $OUT/stamps_c2.txt
echo done
