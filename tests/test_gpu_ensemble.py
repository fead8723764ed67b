"""HIP dynamics-ensemble parity (src/dynamics.py:112-253): _forward1, sample,
_forward_all, compute_loss value + gradients, fit(steps=) and SMBPO.update_models
against the reference's golden fixtures (recorded draws), plus means / mean /
elite_samples / fit(epochs=) against the CPU oracle.

Tolerances (fp32): forward outputs |d| <= 1e-4 + 1e-4*|ref|; gradients
|d| <= 1e-5*max|ref| + 1e-3*|ref| (atomics + different summation order); fit losses
rtol 1e-4; parameters after Adam steps |d| <= 3e-5 + 1e-4*|ref| (as the SAC tests);
elites exact."""
import numpy as np
import pytest
import torch

import drpo_amd
from conftest import load_golden
from gpu_helpers import DEV, COMP, small_smbpo, close
from oracle import drpo_oracle as O

pytestmark = pytest.mark.gpu
ENVS = ['quadrotor', 'tracking', 'cartpole']
PARAM_ATOL, PARAM_RTOL = 3e-5, 1e-4


def model_from(d, env, prefix='sd/'):
    alg = small_smbpo(d, env)
    m = alg.model_ensemble
    sd = {k[len(prefix):]: torch.from_numpy(np.array(d[k])) for k in d.files if k.startswith(prefix)}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    m.state_normalizer.mean.copy_(torch.from_numpy(d['model/norm_mean']))
    m.state_normalizer.std.copy_(torch.from_numpy(d['model/norm_std']))
    return alg, m


def t(x):
    return torch.from_numpy(np.ascontiguousarray(x)).to(DEV)


def check_sd(m, d, prefix, skip=('state_normalizer',)):
    sd = m.state_dict()
    bad = []
    for k in d.files:
        if not k.startswith(prefix):
            continue
        name = k[len(prefix):]
        if name.startswith(skip) or name not in sd:
            continue
        got, exp = sd[name].detach().cpu().numpy(), d[k]
        err = np.abs(got - exp) - (PARAM_ATOL + PARAM_RTOL * np.abs(exp))
        if (err > 0).any():
            bad.append((name, float(np.abs(got - exp).max()), int((err > 0).sum()), exp.size))
    assert not bad, bad[:6]


@pytest.mark.parametrize('env', ENVS)
def test_forward1_sample_forward_all(env):
    d = load_golden(f'ensemble_{env}')
    _, m = model_from(d, env)
    s, a = t(d['in/s']), t(d['in/a'])
    mu, lv = m._forward1(s, a, 1)
    close(mu, d['out/f1_mean'], msg='f1 mean')
    close(lv, d['out/f1_logvar'], msg='f1 logvar')
    m._elite_inds = [1, 3]
    tape = drpo_amd.TapeNoise.from_npz(d, 'sample_tape')
    s2, r = m.sample(s, a, noise=tape)
    assert tape.done()
    close(s2, d['out/sample_s2'], msg='sample s2')
    close(r, d['out/sample_r'], msg='sample r')
    mu, lv = m._forward_all(t(d['in/se']), t(d['in/ae']))
    close(mu, d['out/fall_mean'], msg='all mean')
    close(lv, d['out/fall_logvar'], msg='all logvar')


@pytest.mark.parametrize('env', ENVS)
def test_compute_loss_and_gradients(env):
    d = load_golden(f'ensemble_{env}')
    _, m = model_from(d, env)
    m.optimizer.zero_grad()
    loss = m.compute_loss(t(d['in/loss_s']), t(d['in/loss_a']), t(d['in/loss_t']))
    loss.backward()
    np.testing.assert_allclose(loss.item(), float(d['out/loss']), rtol=1e-5, atol=1e-5)
    params = dict(m.named_parameters())
    bad = []
    for k in d.files:
        if not k.startswith('grad/'):
            continue
        name = k[5:]
        got, exp = params[name].grad.detach().cpu().numpy(), d[k]
        tol = 1e-5 * np.abs(exp).max() + 1e-3 * np.abs(exp)
        if (np.abs(got - exp) > tol).any():
            bad.append((name, float(np.abs(got - exp).max()), float(np.abs(exp).max())))
    assert not bad, bad
    # no-grad call returns the same value and leaves the grads alone
    g0 = m.group.grad.clone()
    with torch.no_grad():
        l2 = m.compute_loss(t(d['in/loss_s']), t(d['in/loss_a']), t(d['in/loss_t']))
    np.testing.assert_allclose(l2.item(), loss.item(), rtol=1e-6)
    assert torch.equal(g0, m.group.grad)


def fill(alg, d):
    rows = {k: t(d['replay/' + k]) for k in COMP}
    half = len(rows['states']) // 2
    alg.replay_buffer.extend(**{k: v[:half] for k, v in rows.items()})
    alg.replay_buffer.extend(**{k: v[half:] for k, v in rows.items()})


@pytest.mark.parametrize('env', ENVS)
def test_fit_steps_matches_reference(env):
    d = load_golden(f'ensemble_{env}')
    alg, m = model_from(d, env)
    fill(alg, d)
    tape = drpo_amd.TapeNoise.from_npz(d, 'fit_tape')
    losses = m.fit(alg.replay_buffer, steps=3, noise=tape)
    assert tape.done()
    np.testing.assert_allclose(losses, d['out/fit_losses'], rtol=1e-4)
    assert m._elite_inds == list(d['out/elite_inds'])
    close(m.state_normalizer.mean, d['fit_sd/state_normalizer.mean'], tol=1e-6, msg='norm mean')
    close(m.state_normalizer.std, d['fit_sd/state_normalizer.std'], tol=1e-6, msg='norm std')
    check_sd(m, d, 'fit_sd/')


@pytest.mark.parametrize('env', ['point-robot', 'quadrotor'])
def test_update_models_matches_reference(env):
    d = load_golden(f'smbpo_update_{env}')
    alg = small_smbpo(d, env)
    sd0 = {k[4:]: torch.from_numpy(np.array(d[k])) for k in d.files if k.startswith('sd0/')}
    sd0.pop('log_alpha', None)
    alg.load_state_dict(sd0, strict=False)
    fill(alg, d)
    tape = drpo_amd.TapeNoise.from_npz(d, 'fit_tape')
    alg.update_models(3, noise=tape)
    assert tape.done()
    assert alg.model_ensemble._elite_inds == list(d['fit/elite_inds'])
    check_sd(alg.model_ensemble, d, 'sd1/model_ensemble.', skip=())


def oracle_params(m):
    return {'m.' + k: v.detach().cpu() for k, v in m.state_dict().items()}


@pytest.mark.parametrize('env', ['quadrotor', 'tracking'])
def test_means_and_elite_samples_vs_oracle(env):
    d = load_golden(f'ensemble_{env}')
    _, m = model_from(d, env)
    P = oracle_params(m)
    E = m.ensemble_size
    s, a = torch.from_numpy(d['in/s']), torch.from_numpy(d['in/a'])
    mu_ref, lv_ref = O.ens_forward_all(P, 'm.', s.repeat(E, 1, 1), a.repeat(E, 1, 1))
    ns, nr = m.means(t(d['in/s']), t(d['in/a']))
    close(ns, mu_ref[:, :, :-1], msg='means s')
    close(nr, mu_ref[:, :, -1], msg='means r')
    ms, mr = m.mean(t(d['in/s']), t(d['in/a']))
    close(ms, mu_ref[:, :, :-1].mean(0), msg='mean s')
    m._elite_inds = [3, 0]
    eps = torch.randn(2, s.shape[0], s.shape[1] + 1)
    tape = drpo_amd.TapeNoise([('randn_like', eps.numpy())])
    es, er = m.elite_samples(t(d['in/s']), t(d['in/a']), noise=tape)
    x = mu_ref[[3, 0]] + torch.exp(lv_ref[[3, 0]]).sqrt() * eps
    close(es, x[:, :, :-1], msg='elite s')
    close(er, x[:, :, -1], msg='elite r')
    # production noise: finite, right shapes, members differ
    es, er = m.elite_samples(t(d['in/s']), t(d['in/a']))
    assert es.shape == (2, s.shape[0], s.shape[1]) and torch.isfinite(es).all()


def test_fit_epochs_vs_oracle():
    """fit(epochs=1) == epochal_training over E epochs of randperm batches (CPU generator)."""
    env = 'quadrotor'
    d = load_golden(f'ensemble_{env}')
    alg, m = model_from(d, env)
    fill(alg, d)
    P = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    buf = {k: v.cpu() for k, v in alg.replay_buffer.get(as_dict=True).items()}   # chronological (may wrap)
    torch.manual_seed(11)
    losses = m.fit(alg.replay_buffer, epochs=1)
    # oracle replay
    torch.manual_seed(11)
    mean, std = O.normalizer_fit(buf['states'])
    P['state_normalizer.mean'], P['state_normalizer.std'] = mean, std
    targets = torch.cat([buf['next_states'], buf['rewards'].unsqueeze(1)], 1)
    keys = O.ens_param_keys(P, '')
    opt = {}
    E, tb, n = m.ensemble_size, m.total_batch_size, len(targets)
    ref_losses = []
    for _ in range(E):
        perm = torch.randperm(n)
        ep = []
        for bi in range(-(-n // tb)):
            idx = perm[bi * tb:(bi + 1) * tb]
            with torch.enable_grad():
                params = {k: P[k].detach().requires_grad_(True) for k in keys}
                Q = dict(P)
                Q.update(params)
                loss = O.ens_compute_loss(Q, '', buf['states'][idx], buf['actions'][idx], targets[idx], E)
                grads = torch.autograd.grad(loss, [params[k] for k in keys])
            ep.append(loss.item())
            for k, g in zip(keys, grads):
                O.adam_update(opt, k, P[k], g.clone(), 1e-3, 1e-4)
        ref_losses.append(float(np.mean(ep)))
    np.testing.assert_allclose(losses, ref_losses, rtol=1e-3)
    sd = m.state_dict()
    for k in keys:
        got, exp = sd[k].cpu().numpy(), P[k].numpy()
        # many Adam steps: compare loosely (fp32 summation order drifts through Adam)
        assert np.abs(got - exp).max() <= 2e-3 + 1e-2 * np.abs(exp).max(), k


@pytest.mark.parametrize('env', ['quadrotor', 'tracking'])
def test_fit_epochs_matches_reference_fixture(env):
    """fit(epochs=1) against the reference's own run (src/dynamics.py:185-194 ->
    src/train.py::epochal_training: E epochs of torch.randperm batches, the last one
    ragged, recorded by make_golden.py with the CPU generator re-seeded right before the
    call). Per-element parameter tolerance as the other fit tests."""
    d = load_golden(f'fit_epochs_{env}')
    alg, m = model_from(d, env)
    fill(alg, d)
    torch.manual_seed(int(d['torch_seed']))
    losses = m.fit(alg.replay_buffer, epochs=1)
    assert len(losses) == len(d['out/losses']) == m.ensemble_size
    np.testing.assert_allclose(losses, d['out/losses'], rtol=1e-4)
    close(m.state_normalizer.mean, d['model/norm_mean'], tol=1e-6, msg='normalizer mean')
    close(m.state_normalizer.std, d['model/norm_std'], tol=1e-6, msg='normalizer std')
    check_sd(m, d, 'fit_sd/')


def test_fit_production_noise():
    """Device (Philox) minibatch indices: loss goes down over steps, elites are distinct
    members, parameters stay finite."""
    env = 'quadrotor'
    d = load_golden(f'ensemble_{env}')
    alg, m = model_from(d, env)
    fill(alg, d)
    losses = m.fit(alg.replay_buffer, steps=60)
    assert len(losses) == 60 and np.isfinite(losses).all()
    assert np.mean(losses[-10:]) < np.mean(losses[:10])
    assert len(set(m._elite_inds)) == m.num_elites and all(0 <= i < m.ensemble_size for i in m._elite_inds)
    assert torch.isfinite(m.group.data).all()
