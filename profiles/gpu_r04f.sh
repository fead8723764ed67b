# kernel floor probe: kernarg size / read pattern / memory chain
OUT=gpurun_out/r04f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 ./profiles/karg_probe > $OUT/karg_probe.txt 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- ./profiles/karg_probe > $OUT/karg_prof.log 2>&1 || exit 1
echo done
