# round 4: 4x4-block optimizer (probe, tests), weight-gradient ring depth A/B, bench
OUT=gpurun_out/r04d
mkdir -p $OUT
export TMPDIR=/tmp
LIBD=$PWD/distributional-reachability-policy-optimization_amd
timeout -k 10 180 python -u profiles/optim_probe.py > $OUT/optim_probe.json 2> $OUT/optim_probe.err || exit 1
timeout -k 10 120 python -u -m pytest tests/test_gpu_optim.py -x -q --timeout 60 --timeout-method thread > $OUT/optim_test.log 2>&1 || { echo optim test failed; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1 || { echo pytest failed; exit 1; }
DRPO_WGRAD_PER_CU=2 timeout -k 10 120 python -u profiles/wgrad_probe.py >> $OUT/wgrad_probe.jsonl 2>> $OUT/wgrad_probe.err || exit 1
for v in wgd2 wgd4 wgd5; do DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_$v.so timeout -k 10 120 python -u profiles/wgrad_probe.py | sed "s/^{/{\"lib\": \"$v\", /" >> $OUT/wgrad_probe.jsonl 2>> $OUT/wgrad_probe.err || exit 1; done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit 1
echo done
