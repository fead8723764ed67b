# round 4: optimizer + weight-gradient probes (ring depth, residency, phase stamps), bench
OUT=gpurun_out/r04c
mkdir -p $OUT
export TMPDIR=/tmp
LIBD=$PWD/distributional-reachability-policy-optimization_amd
timeout -k 10 180 python -u profiles/optim_probe.py > $OUT/optim_probe.json 2> $OUT/optim_probe.err || exit 1
for pc in 1 2; do DRPO_WGRAD_PER_CU=$pc timeout -k 10 120 python -u profiles/wgrad_probe.py >> $OUT/wgrad_probe.jsonl 2>> $OUT/wgrad_probe.err || exit 1; done
for v in wgd8 wgd3; do DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_$v.so timeout -k 10 120 python -u profiles/wgrad_probe.py | sed "s/^{/{\"lib\": \"$v\", /" >> $OUT/wgrad_probe.jsonl 2>> $OUT/wgrad_probe.err || exit 1; done
for v in stamps stamps_wgd8; do DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_$v.so timeout -k 10 120 python -u profiles/wgrad_probe.py | sed "s/^{/{\"lib\": \"$v\", /" >> $OUT/wgrad_probe.jsonl 2>> $OUT/wgrad_probe.err || exit 1; done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit 1
echo done
