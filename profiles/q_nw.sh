set -e
OUT=gpurun_out/nw
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_sac.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest8.log 2>&1
DRPO_ROLLOUT_NW=16 timeout -k 10 200 python -u -m pytest tests/test_gpu_rollout.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest16.log 2>&1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-fit > $OUT/b8.json 2> $OUT/b8.err
DRPO_ROLLOUT_NW=16 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-fit > $OUT/b16.json 2> $OUT/b16.err
echo ok
