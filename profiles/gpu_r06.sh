#!/bin/bash
# Round-6 GPU pass: full GPU suite, smoke, default bench line and the SAC per-launch
# micro-run. Usage: bash profiles/gpu_r06.sh <tag> [skip-tests]
OUT=gpurun_out/${1:-r06}
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rf -x > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc $rc" >> $OUT/pytest_gpu.log; tail -2 $OUT/pytest_gpu.log
  [ $rc -eq 0 ] || exit 1
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 180 python -u profiles/sac_micro.py --steps 10 > $OUT/sac_micro.json 2> $OUT/sac_micro.err || exit 1
python profiles/summ.py $OUT/bench.json $OUT/sac_micro.json
