"""Multi-process (gloo, world_size 2 and 4) CPU tests of the data-parallel path."""
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize('world', [2, 4])
def test_gloo_data_parallel_plumbing(world):
    port = _port()
    env0 = {k: v for k, v in os.environ.items() if k not in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK')}
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, 'dist_cpu_worker.py')],
                              env=dict(env0, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR='127.0.0.1',
                                       MASTER_PORT=str(port), CUDA_VISIBLE_DEVICES=''),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(world)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=300)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, out))
    for rc, out in outs:
        assert rc == 0, out[-3000:]
