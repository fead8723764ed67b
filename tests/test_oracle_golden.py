"""Pin the CPU oracle against golden vectors produced by the reference itself
(tests/golden/make_golden.py). Bit-exact at 4 threads unless stated."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import drpo_oracle as O


def sd(d, prefix, strip=''):
    out = {}
    for k in d.files:
        if k.startswith(prefix):
            key = k[len(prefix):]
            if strip and key.startswith(strip):
                key = key[len(strip):]
            out[key] = torch.from_numpy(np.array(d[k]))
    return out


def assert_same(a, b, exact=True, atol=0.0, rtol=0.0, msg=''):
    a = a.detach().numpy() if torch.is_tensor(a) else np.asarray(a)
    b = b.detach().numpy() if torch.is_tensor(b) else np.asarray(b)
    assert a.shape == b.shape, (msg, a.shape, b.shape)
    if exact:
        assert np.array_equal(a, b), (msg, np.abs(a.astype(np.float64) - b).max())
    else:
        np.testing.assert_allclose(a, b, atol=atol, rtol=rtol, err_msg=msg)


@pytest.mark.parametrize('env', ['point-robot', 'quadrotor', 'cartpole', 'tracking'])
def test_constraints(env):
    d = load_golden('constraints')
    s = d[f'{env}/states']
    done, viol, h = O.ENV_CONSTRAINTS[env](s)
    np.testing.assert_array_equal(viol, d[f'{env}/violation'])
    href = d[f'{env}/h']
    href = href[:, None] if href.ndim == 1 else href
    np.testing.assert_allclose(h, href, rtol=0, atol=1e-6 if env == 'tracking' else 0)
    if env != 'quadrotor':          # quadrotor out-of-bound thresholds: parity unpinned
        np.testing.assert_array_equal(done, d[f'{env}/done'])


@pytest.mark.parametrize('env', ['quadrotor', 'tracking', 'cartpole'])
def test_ensemble(env):
    d = load_golden(f'ensemble_{env}')
    P = sd(d, 'sd/')
    E = int(d['meta/E'])
    P['state_normalizer.mean'] = torch.from_numpy(d['model/norm_mean'])
    P['state_normalizer.std'] = torch.from_numpy(d['model/norm_std'])
    s, a = torch.from_numpy(d['in/s']), torch.from_numpy(d['in/a'])
    with torch.no_grad():
        mu, lv = O.ens_forward1(P, '', s, a, 1)
    assert_same(mu, d['out/f1_mean'], msg='f1 mean')
    assert_same(lv, d['out/f1_logvar'], msg='f1 logvar')
    rng = O.TapeRNG.from_npz(d, 'sample_tape')
    with torch.no_grad():
        s2, r = O.ens_sample(P, '', s, a, [1, 3], rng)
    assert rng.done()
    assert_same(s2, d['out/sample_s2'])
    assert_same(r, d['out/sample_r'])
    with torch.no_grad():
        mu, lv = O.ens_forward_all(P, '', torch.from_numpy(d['in/se']), torch.from_numpy(d['in/ae']))
    assert_same(mu, d['out/fall_mean'])
    assert_same(lv, d['out/fall_logvar'])
    keys = O.ens_param_keys(P, '')
    params = {k: P[k].clone().requires_grad_(True) for k in keys}
    Q = dict(P)
    Q.update(params)
    loss = O.ens_compute_loss(Q, '', torch.from_numpy(d['in/loss_s']), torch.from_numpy(d['in/loss_a']),
                              torch.from_numpy(d['in/loss_t']), E)
    loss.backward()
    assert_same(loss, d['out/loss'])
    for k in keys:
        assert_same(params[k].grad, d['grad/' + k], msg=k)


def test_ensemble_fit():
    d = load_golden('ensemble_quadrotor')
    P = sd(d, 'sd/')
    cap = int(d['meta/buffer_max'])
    S, A, C = int(d['meta/S']), int(d['meta/A']), int(d['meta/C'])
    buf = O.RingBuffer(S, A, C, cap)
    rows = {k: torch.from_numpy(d['replay/' + k]) for k in O.COMPONENTS}
    half = len(rows['states']) // 2
    buf.extend({k: v[:half] for k, v in rows.items()})
    buf.extend({k: v[half:] for k, v in rows.items()})
    chrono = {k: buf.get(k) for k in O.COMPONENTS}
    rng = O.TapeRNG.from_npz(d, 'fit_tape')
    losses, elites = O.ens_fit(P, '', {}, chrono, 3, int(d['meta/E']), int(d['meta/model_batch']),
                               int(d['meta/model_batch']), int(d['meta/num_elites']), rng)
    assert rng.done()
    np.testing.assert_array_equal(np.array(losses), d['out/fit_losses'])
    assert elites == list(d['out/elite_inds'])
    for k, v in sd(d, 'fit_sd/').items():
        assert_same(P[k], v, msg=k)


@pytest.mark.parametrize('env', ['quadrotor', 'tracking'])
def test_ensemble_fit_epochs(env):
    """fit(epochs=1) -> epochal_training, pinned bit-exactly to the reference's run."""
    d = load_golden(f'fit_epochs_{env}')
    P = sd(d, 'sd/')
    cap = int(d['meta/buffer_max'])
    S, A, C = int(d['meta/S']), int(d['meta/A']), int(d['meta/C'])
    buf = O.RingBuffer(S, A, C, cap)
    rows = {k: torch.from_numpy(d['replay/' + k]) for k in O.COMPONENTS}
    half = len(rows['states']) // 2
    buf.extend({k: v[:half] for k, v in rows.items()})
    buf.extend({k: v[half:] for k, v in rows.items()})
    chrono = {k: buf.get(k) for k in O.COMPONENTS}
    torch.manual_seed(int(d['torch_seed']))
    losses = O.ens_fit_epochs(P, '', {}, chrono, 1, int(d['meta/E']), int(d['meta/model_batch']))
    np.testing.assert_array_equal(np.array(losses), d['out/losses'])
    for k, v in sd(d, 'fit_sd/').items():
        assert_same(P[k], v, msg=k)


@pytest.mark.parametrize('tag', ['point-robot', 'quadrotor', 'fullwidth_quad'])
def test_rollout(tag):
    """fullwidth_quad: the reference's default widths (actor 256, model 200, E = 7)."""
    d = load_golden(f'rollout_{tag}')
    env = str(d['meta/env'])
    full = sd(d, 'sd/')
    P = {k[len('solver.'):]: v for k, v in full.items() if k.startswith('solver.actor.')}
    P.update({k: v for k, v in full.items() if k.startswith('model_ensemble.')})
    P['model_ensemble.state_normalizer.mean'] = torch.from_numpy(d['model/norm_mean'])
    P['model_ensemble.state_normalizer.std'] = torch.from_numpy(d['model/norm_std'])
    S, A, C = int(d['meta/S']), int(d['meta/A']), int(d['meta/C'])
    buf = O.RingBuffer(S, A, C, int(d['meta/buffer_max']))
    rows = {k: torch.from_numpy(d['replay/' + k]) for k in O.COMPONENTS}
    half = len(rows['states']) // 2
    buf.extend({k: v[:half] for k, v in rows.items()})
    buf.extend({k: v[half:] for k, v in rows.items()})
    rng = O.TapeRNG.from_npz(d, 'tape')
    out = O.rollout(P, 'actor.net.', 'model_ensemble.', list(d['model/elite_inds']), buf.get('states'), env,
                    int(d['meta/B']), int(d['meta/H']), rng)
    assert rng.done()
    assert len(out['states']) == int(d['out/n'])
    for k in O.COMPONENTS:
        assert_same(out[k], d['out/' + k], msg=k)


def ssac_cfg(d):
    c = dict(batch_size=int(d['meta/sac_batch']), distributional=bool(d['meta/distributional']),
             uncertainty=bool(d['meta/uncertainty']), target_entropy=-2.0, penalty_lb=-1.0,
             actor_lr=1e-4, updates_per_training=1 * 2 * 10)
    for k in d.files:                  # solver-flag fixtures (make_golden.SOLVER_FLAG_CASES)
        if k.startswith('flag/'):
            c[k[len('flag/'):]] = d[k].item()
    return c


SSAC_TAGS = ['drpo_point', 'drpo_quad', 'vanilla_quad', 'robust_quad', 'robust_point', 'scalar_mult_point',
             'scalar_mult_quad', 'fixed_alpha_quad', 'log_alpha_point', 'cost_point', 'cost_quad',
             'fullwidth_quad']   # the reference's default widths (256): make_golden.gen_fullwidth


@pytest.mark.parametrize('tag', SSAC_TAGS)
def test_ssac_updates(tag):
    d = load_golden(f'ssac_{tag}')
    P0 = sd(d, 'sd0/')
    C, A = int(d['meta/C']), int(d['meta/A'])
    cfg = ssac_cfg(d)
    if 'model/elite_inds' in d.files:
        cfg.update(elites=list(d['model/elite_inds']), env=str(d['meta/env']))
    orc = O.SSACOracle(P0, cfg, C, A)
    batch = [torch.from_numpy(d['in/' + k]) for k in ['s', 'a', 's2', 'r', 'd', 'v', 'h']]
    rng = O.TapeRNG.from_npz(d, 'critic_tape')
    lq, lqc = orc.update_critic(*batch, rng)
    assert rng.done()
    assert_same(lq, d['out/lq'])
    assert_same(lqc, d['out/lqc'])
    for k, v in sd(d, 'sd1/').items():
        if not k.startswith('model_ensemble') and k != 'total_updates':
            assert_same(orc.P[k], v, msg='after critic ' + k)
    rng = O.TapeRNG.from_npz(d, 'actor_tape')
    orc.update_actor_and_alpha(batch[0], rng)
    assert rng.done()
    for k, v in sd(d, 'sd2/').items():
        if k == 'log_alpha':
            assert_same(orc.log_alpha, v)
        elif not k.startswith('model_ensemble') and k != 'total_updates':
            assert_same(orc.P[k], v, msg='after actor ' + k)
    rng = O.TapeRNG.from_npz(d, 'mult_tape')
    orc.update_multiplier(batch[0], rng)
    assert rng.done()
    for k, v in sd(d, 'sd3/').items():
        if not k.startswith('model_ensemble') and k != 'total_updates':
            assert_same(orc.P[k], v, msg='after multiplier ' + k)
    lrs = [orc.sched[g].lr for g in ['critic', 'actor', 'actor_safe', 'multiplier']]
    np.testing.assert_array_equal(np.array(lrs), d['lr3'])


def smbpo_cfg(d):
    c = ssac_cfg(d)
    return dict(B=int(d['meta/B']), H=int(d['meta/H']), buffer_max=int(d['meta/buffer_max']), real_fraction=0.1,
                reward_scale=2.0, alive_bonus=2.0, constraint_scale=10.0, constraint_offset=0.5,
                solver_updates_per_step=10, sac=c,
                model=dict(E=int(d['meta/E']), batch_size=int(d['meta/model_batch']),
                           holdout=int(d['meta/model_batch']), num_elites=int(d['meta/num_elites'])))


@pytest.mark.parametrize('tag', ['point-robot', 'quadrotor', 'cost_point'])
def test_smbpo_update(tag):
    d = load_golden(f'smbpo_update_{tag}')
    env = str(d['meta/env'])
    full = sd(d, 'sd0/')
    la = full.pop('log_alpha')
    full['solver.log_alpha'] = la
    S, A, C = int(d['meta/S']), int(d['meta/A']), int(d['meta/C'])
    orc = O.SMBPOOracle(full, env, smbpo_cfg(d), S, A, C)
    rows = {k: torch.from_numpy(d['replay/' + k]) for k in O.COMPONENTS}
    half = len(rows['states']) // 2
    orc.replay.extend({k: v[:half] for k, v in rows.items()})
    orc.replay.extend({k: v[half:] for k, v in rows.items()})
    rng = O.TapeRNG.from_npz(d, 'fit_tape')
    orc.update_models(3, rng)
    assert rng.done()
    assert orc.elite_inds == list(d['fit/elite_inds'])
    for r in range(2):
        rng = O.TapeRNG.from_npz(d, f'rau{r}_tape')
        orc.rollout_and_update(rng)
        assert rng.done()
    assert len(orc.virt) == int(d['virt/n'])
    for k in O.COMPONENTS:
        assert_same(orc.virt.get(k), d['virt/' + k], msg=k)
    for k, v in sd(d, 'sd2/').items():
        if k == 'log_alpha':
            assert_same(orc.ssac.log_alpha, v)
        elif k.startswith('solver.') and not k.startswith('solver.model_ensemble') and k != 'solver.total_updates':
            assert_same(orc.ssac.P[k[len('solver.'):]], v, msg=k)
        elif k.startswith('model_ensemble.'):
            assert_same(orc.M[k], v, msg=k)
    np.testing.assert_array_equal(np.array([float(x) for x in orc.critic_losses]), d['losses/critic'])
