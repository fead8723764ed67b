set -e
mkdir -p gpurun_out/g2
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_ensemble.py -x -v --timeout 240 --timeout-method thread > gpurun_out/g2/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/g2/bench.json 2> gpurun_out/g2/bench.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 4 --warmup 1 --backend gloo --no-cpu-baseline > gpurun_out/g2/bench2.json 2> gpurun_out/g2/bench2.err
echo done
