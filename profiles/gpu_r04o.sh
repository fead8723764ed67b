OUT=gpurun_out/r04o
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad.py tests/test_gpu_optim.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo tests failed; exit 1; }
echo done
