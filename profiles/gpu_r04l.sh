# weight-gradient planner: minimum rows per unit A/B (probe)
OUT=gpurun_out/r04l
mkdir -p $OUT
export TMPDIR=/tmp
for mr in 0 512 1024 2048; do DRPO_WGRAD_MIN_ROWS=$mr timeout -k 10 120 python -u profiles/wgrad_probe.py >> $OUT/wgrad_probe.jsonl 2>> $OUT/wgrad_probe.err || exit 1; done
for mr in 0 1024; do DRPO_WGRAD_MIN_ROWS=$mr timeout -k 10 120 python -u profiles/wgrad_probe.py >> $OUT/wgrad_probe.jsonl 2>> $OUT/wgrad_probe.err || exit 1; done
echo done
