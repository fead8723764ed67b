#!/bin/bash
# round-3 pass: full GPU suite (new parity tests), smoke, config-1 bench line, traffic
# passes on this build for configs 2-5, default bench line.
OUT=gpurun_out/r03b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --maxfail=30 --timeout 400 --timeout-method thread -rf > $OUT/pytest.log 2>&1
echo "pytest rc $?" >> $OUT/pytest.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config 1 --no-cpu-baseline > $OUT/bench_c1.json 2> $OUT/bench_c1.err || exit 1
bash profiles/traffic_configs.sh r03b 2 3 4 5 || exit 1
echo done
