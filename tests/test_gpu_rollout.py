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


@pytest.mark.parametrize('tag', ['point-robot', 'quadrotor', 'fullwidth_quad'])
def test_rollout_matches_reference_fixture(tag):
    """fullwidth_quad: the reference's default widths (actor 256, model 200, E = 7), B = 64,
    H = 2: the production persist kernel's LDS-resident actor and paired-heads paths."""
    d = load_golden(f'rollout_{tag}')
    env = str(d['meta/env'])
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


def _full_width_case(env, B, H):
    """SMBPO at default widths + a replay of N states, and the oracle's rollout
    driven by live reference RNG calls (returns alg, oracle output, recorded draws)."""
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
    return alg, ref, live.entries


FULL_WIDTH = [('quadrotor', 4096, 10), ('point-robot', 1024, 20), ('tracking', 512, 8), ('cartpole', 256, 5)]


@pytest.mark.parametrize('env,B,H', FULL_WIDTH)
def test_rollout_matches_oracle_full_width(env, B, H):
    """Default widths (actor 256, model 200, E=7) at BASELINE-like shapes vs the oracle
    driven by the live reference RNG calls; the recorded draws are fed to the HIP path
    (compacted per-step draws -> the per-step engine)."""
    alg, ref, entries = _full_width_case(env, B, H)
    out = alg.rollout(alg.actor, noise=drpo_amd.TapeNoise(entries))
    torch.cuda.synchronize()
    n = len(ref['states'])
    assert len(out) == n
    got = out.get(as_dict=True)
    for k in COMP:
        close(got[k], ref[k], tol=2e-4, msg=k)


def original_row_tape(entries, ref, B):
    """Re-index the reference's per-step draws (row k of step t = k-th surviving row)
    by original batch row: step t's arrays become [B, dim], row i = trajectory i
    (zeros for rows already done). Survivors follow from the oracle's dones:
    step t+1 keeps step t's rows with done == 0, in order (src/smbpo.py:243-246)."""
    ids = np.arange(B)
    out, off, t_rows = [], 0, None
    dones = np.asarray(ref['dones']).astype(bool)
    for kind, v in entries:
        if kind == 'normal':               # eps_a of a step: [n_t, A]
            n = v.shape[0]
            assert n == len(ids)
            full = np.zeros((B, v.shape[1]), np.float32)
            full[ids] = v
            out.append((kind, full))
            t_rows = n
        elif kind == 'randn_like':         # eps_m of the same step: [n_t, S+1]
            full = np.zeros((B, v.shape[1]), np.float32)
            full[ids] = v
            out.append((kind, full))
            ids = ids[~dones[off:off + t_rows]]
            off += t_rows
        else:
            out.append((kind, v))
    assert off == len(dones)
    return out


def test_fused_engine_matches_reference_fixture_full_width():
    """The production fused-horizon engine (rollout_persist_kernel: LDS-resident actor,
    member layer-1 prefetch, 13-block split, paired 200-wide heads) against the
    reference-held full-width vector (rollout_fullwidth_quad: actor 256, model 200,
    E = 7, B = 64, H = 2), the recorded draws re-indexed by original row."""
    from drpo_amd import ops
    d = load_golden('rollout_fullwidth_quad')
    alg = small_smbpo(d, 'quadrotor')
    load_sd(alg, d, 'sd/')
    fill_replay(alg, d)
    m = alg.model_ensemble
    m.state_normalizer.mean.copy_(torch.from_numpy(d['model/norm_mean']))
    m.state_normalizer.std.copy_(torch.from_numpy(d['model/norm_std']))
    m._elite_inds = list(d['model/elite_inds'])
    entries = drpo_amd.TapeNoise.from_npz(d, 'tape').entries
    tape = drpo_amd.TapeNoise(original_row_tape(entries, {'dones': d['out/dones']}, alg.rollout_batch_size))
    alg.rollout_engine = 2
    out = ops.rollout(alg, alg.actor, None, tape, eps_layout=1)
    torch.cuda.synchronize()
    assert tape.done() and len(out) == int(d['out/n'])
    got = alg.virt_buffer.get(as_dict=True)
    for k in COMP:
        close(got[k], d['out/' + k], tol=2e-4, msg=k)


@pytest.mark.parametrize('env,B,H', FULL_WIDTH)
def test_fused_engine_matches_oracle_full_width(env, B, H):
    """The fused-horizon engine (production default) against the same oracle run,
    its recorded draws re-indexed by original row (rows die in these cases, so the
    tile masking, per-(step, tile) counts and the ordered emit are all exercised)."""
    alg, ref, entries = _full_width_case(env, B, H)
    tape = drpo_amd.TapeNoise(original_row_tape(entries, ref, B))
    from drpo_amd import ops
    out = ops.rollout(alg, alg.actor, None, tape, eps_layout=1)
    torch.cuda.synchronize()
    assert tape.done()
    n = len(ref['states'])
    assert len(out) == n
    assert len(alg.virt_buffer) == n
    got = out.get(as_dict=True)
    for k in COMP:
        close(got[k], ref[k], tol=2e-4, msg=k)


@pytest.mark.parametrize('B,H,rpt', [(4096, 10, 0), (1000, 7, 0), (8192, 4, 32), (8192, 3, 16)])
def test_fused_engine_matches_step_engine_device_noise(B, H, rpt):
    """Production noise (Philox keyed by row and step): with no row finishing the two
    engines draw identical numbers, so their buffers must agree to rounding (bench
    workload in steady mode, plus ragged and 32-row-tile shapes)."""
    import random
    import bench
    outs = []
    for engine in (1, 2):
        random.seed(11)
        alg = bench.make_alg(DEV, B, H, 7, 0, bench.QUAD_JSON)
        rep = bench.synth_replay('quadrotor', 20000, np.random.RandomState(0))
        alg.replay_buffer.extend(**{k: torch.from_numpy(v).to(DEV) for k, v in rep.items()})
        alg.model_ensemble.state_normalizer.fit(alg.replay_buffer.get('states'))
        bench.steady_mode(alg)
        alg.rollout_engine, alg.rows_per_tile = engine, rpt
        out = alg.rollout(alg.actor, noise=drpo_amd.DeviceNoise(1234))
        torch.cuda.synchronize()
        assert len(out) == B * H
        outs.append(out.get(as_dict=True))
    for k in COMP:
        a, b = outs[0][k], outs[1][k]
        if a.dtype == torch.bool:
            assert torch.equal(a, b), k
        else:
            close(a, b, tol=1e-5, msg=k)


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


def _prod_alg(seed):
    cfg = drpo_amd.SMBPO.Config()
    cfg.update({'horizon': 5, 'rollout_batch_size': 2048, 'buffer_max': 50000})
    torch.manual_seed(3)
    alg = drpo_amd.SMBPO(cfg, lambda id=None: ENVS['quadrotor'](), None, 1, device=DEV, noise_seed=seed)
    N = 8000
    g = torch.Generator(device='cpu').manual_seed(11)
    s = torch.randn(N, 12, generator=g).to(DEV)
    s[:, 2] = s[:, 2].abs() * 0.2 + 0.6
    z = lambda *sh, dt=torch.float32: torch.zeros(*sh, dtype=dt, device=DEV)
    alg.replay_buffer.extend(states=s, actions=z(N, 2), next_states=s, rewards=z(N), dones=z(N, dt=torch.bool),
                             violations=z(N, dt=torch.bool), constraint_values=z(N, 2))
    alg.model_ensemble.state_normalizer.fit(s)
    alg.model_ensemble._elite_inds = [0, 1, 2, 3, 4]
    return alg


def test_device_noise_seed_controls_rollout_draws():
    """the production noise key follows the seed -- the same seed (on fresh,
    identically initialised trainers) reproduces the rollout bit for bit, another seed
    draws different initial states and noise."""
    a1, a2, b = _prod_alg(101), _prod_alg(101), _prod_alg(202)
    r1, r2, r3 = (x.rollout(x.actor).get(as_dict=True) for x in (a1, a2, b))
    for k in COMP:
        assert torch.equal(r1[k], r2[k]), k
    assert not torch.equal(r1['states'][:2048], r3['states'][:2048])
    assert not torch.equal(r1['actions'][:2048], r3['actions'][:2048])


@pytest.mark.parametrize('high,size', [(10, 10), (1000, 37), (100000, 4096), (5, 0)])
def test_buffer_sample_without_replacement(high, size):
    """SampleBuffer.sample(replace=False) (src/sampling.py:147-151): distinct in-range rows."""
    from drpo_amd.buffers import SampleBuffer
    buf = SampleBuffer(3, 2, high, device=DEV)
    st = torch.arange(high, dtype=torch.float32, device=DEV)[:, None].repeat(1, 3)
    z = lambda *sh, dt=torch.float32: torch.zeros(*sh, dtype=dt, device=DEV)
    buf.extend(states=st, actions=z(high, 2), next_states=st, rewards=z(high), dones=z(high, dt=torch.bool))
    (s, *_), idx = buf.sample(size, replace=False, device=DEV, include_indices=True)
    assert idx.shape == (size,) and torch.unique(idx).numel() == size
    if size:
        assert int(idx.min()) >= 0 and int(idx.max()) < high
    assert torch.equal(s[:, 0].long(), idx)
    with pytest.raises(ValueError):
        buf.sample(high + 1, replace=False, device=DEV)


def test_cartpole_threshold_follows_env():
    """the cartpole constraint uses the env's own threshold
    (src/env/poles/inverted_pendulum.py:11-17), not the default 0.2."""
    from drpo_amd import envs, ops

    class SafeInvertedPendulumEnv:
        x_threshold, th_threshold = 0.9, 0.35
    p = envs.device_env_params(SafeInvertedPendulumEnv())
    assert p['env_id'] == 2 and p['thr1'] == 0.35
    s = torch.randn(513, 4, device=DEV)
    done, viol, h = ops.env_constraints(p, s)
    x, t = s[:, 0].double(), s[:, 1].double()
    ref = torch.stack([-x - 0.9, -t - 0.35, x - 0.9, t - 0.35], 1)
    assert torch.equal(h, ref.float())
    assert torch.equal(viol, (ref > 0).any(1)) and torch.equal(done, viol)


def test_rollout_host_env_fallback_matches_reference_fixture():
    """An env class the build has no device constraint functions for (not in
    envs.ENV_IDS) keeps the reference's host round trip (ops.rollout_host_env: HIP
    policy + member sample, the env's own numpy check_done / check_violation /
    get_constraint_values each step). Same reference fixture as the device path."""
    import drpo_amd
    from drpo_amd.envs import device_env_params
    from pr_env import PointRobot

    class HostOnlyPointRobot(PointRobot):     # unknown class name -> no device fns
        pass

    d = load_golden('rollout_point-robot')
    alg = small_smbpo(d, 'point-robot', factory=lambda id=None: HostOnlyPointRobot())
    assert alg.env_params is None and device_env_params(alg.real_env) is None
    load_sd(alg, d, 'sd/')
    fill_replay(alg, d)
    m = alg.model_ensemble
    m.state_normalizer.mean.copy_(torch.from_numpy(d['model/norm_mean']))
    m.state_normalizer.std.copy_(torch.from_numpy(d['model/norm_std']))
    m._elite_inds = list(d['model/elite_inds'])
    tape = drpo_amd.TapeNoise.from_npz(d, 'tape')
    alg.rollout(alg.actor, noise=tape)
    torch.cuda.synchronize()
    assert tape.done()
    n = int(d['out/n'])
    assert len(alg.virt_buffer) == n
    got = alg.virt_buffer.get(as_dict=True)
    for k in COMP:
        close(got[k], d['out/' + k], msg=k)
