"""Data-parallel SAC update on the GPU: 2 ranks (child processes sharing the one
MI355X, gloo for the exchange) each take half of the golden batch; the
all-reduced result must equal the single-process reference result."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize('tag', ['drpo_quad', 'robust_point', 'scalar_mult_point', 'log_alpha_point'])
def test_sac_data_parallel_two_ranks(tag):
    port = _port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE='2', LOCAL_RANK=str(r), MASTER_ADDR='127.0.0.1',
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY='0')
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, 'dp_worker.py'), tag, 'gloo'], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, out))
    for rc, out in outs:
        assert rc == 0, out[-3000:]


def _run_ranks(script, args, world=2):
    port = _port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR='127.0.0.1',
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY='0')
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, script)] + args, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, out))
    bad = [f'--- rank {r} (rc {rc}) ---\n{out[-2500:]}' for r, (rc, out) in enumerate(outs) if rc != 0]
    assert not bad, '\n'.join(bad)


@pytest.mark.parametrize('env', ['quadrotor', 'tracking'])
def test_member_sharded_fit_two_ranks(env):
    """SURVEY §8(e) model fit: members sharded over 2 ranks reproduce the
    single-process reference fit (all members, losses, elites) on every rank."""
    _run_ranks('fit_shard_worker.py', [env])


def test_device_noise_replicas_stay_identical():
    """production DP with per-rank Philox streams and shared host choices
    keeps every replica's parameters identical (2 ranks, gloo, one GPU)."""
    _run_ranks('dp_noise_worker.py', [])


def test_member_sharded_fit_e8_four_ranks(tmp_path):
    """Config 4's ensemble split (E=8 over 4 ranks) vs the same fit in one process."""
    import numpy as np
    import torch
    import drpo_amd
    sys.path.insert(0, HERE)
    import shard8_worker as w
    alg = w.build(torch.device('cuda', 0))
    m = alg.model_ensemble
    losses = m.fit(alg.replay_buffer, steps=3,
                   noise=drpo_amd.TapeNoise(w.tape(3, len(alg.replay_buffer), 8 * 256, 256)))
    torch.cuda.synchronize()
    out = str(tmp_path / 'ref.npz')
    np.savez(out, losses=np.array(losses), elites=np.array(m._elite_inds), params=w.flat_params(m))
    _run_ranks('shard8_worker.py', [out], world=4)


def test_bench_two_ranks_gloo():
    """Regression test for the N>1 bench path (round-1 hang: a post-pass on rank 0 only
    while the updates all-reduce): bench.py under torchrun, 2 ranks on the one GPU
    with gloo for the exchange, must finish and print one JSON line."""
    import json
    port = _port()
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2', '--master-addr',
           '127.0.0.1', '--master-port', str(port), os.path.join(os.path.dirname(HERE), 'bench.py'), '--gpus', '2',
           '--backend', 'gloo', '--steps', '2', '--warmup', '1', '--fit-steps', '2', '--no-cpu-baseline']
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY='0')
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-3000:])
    lines = [x for x in p.stdout.splitlines() if x.startswith('{')]
    assert len(lines) == 1, p.stdout[-2000:]
    res = json.loads(lines[0])
    assert res['n_gpus'] == 2 and res['value'] > 0 and res['sac']['value'] > 0
    assert res['model_fit']['sharding'].startswith('members')


def test_bench_gpus_flag_launches_ranks():
    """a plain `bench.py --gpus 2` (no torchrun wrapper) starts the 2
    ranks itself and prints rank 0's single line with n_gpus 2."""
    import json
    cmd = [sys.executable, os.path.join(os.path.dirname(HERE), 'bench.py'), '--gpus', '2', '--backend', 'gloo',
           '--steps', '2', '--warmup', '1', '--fit-steps', '2', '--no-cpu-baseline']
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-3000:])
    lines = [x for x in p.stdout.splitlines() if x.strip()]
    assert len(lines) == 1, p.stdout[-2000:]
    res = json.loads(lines[0])
    assert res['n_gpus'] == 2 and res['config']['parallelism'] == 'dp2'
    assert res['value'] > 0 and res['sac']['value'] > 0
    assert res['model_fit']['sharding'].startswith('members')


@pytest.mark.parametrize('mode', ['batch', 'members'])
def test_dp_collection_replicas_agree(mode):
    """step_generator past buffer_min + model fits under DP (2 ranks, gloo,
    one GPU, torch seeded per rank): the real replay, normalizer, reward bounds,
    elites and parameters agree on every rank; the imagined rollouts do not."""
    _run_ranks('dp_collect_worker.py', [mode])
