# round 4: new weight-gradient kernel -- its own test, the SAC / fit parity tests, smoke, bench
OUT=gpurun_out/r04b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad.py -x -v --timeout 120 --timeout-method thread > $OUT/wgrad_test.log 2>&1 || { echo wgrad test failed; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1
echo "pytest rc $?" >> $OUT/pytest_gpu.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python bench.py --no-cpu-baseline > $OUT/stats.log 2>&1 || exit 1
for pc in 1 2 3 4; do DRPO_WGRAD_PER_CU=$pc timeout -k 10 120 python -u profiles/wgrad_probe.py >> $OUT/wgrad_probe.jsonl 2>> $OUT/wgrad_probe.err || exit 1; done
DRPO_LIB_OVERRIDE=$PWD/distributional-reachability-policy-optimization_amd/libdrpo_hip_stamps.so timeout -k 10 120 python -u profiles/wgrad_probe.py >> $OUT/wgrad_probe_stamps.jsonl 2>> $OUT/wgrad_probe.err || exit 1
echo done
