"""Stand-alone network forwards used outside the fused SAC step (real-env acting,
evaluation, diagnostics): SquashedGaussianPolicy.act / distr, CriticEnsemble.all /
min / mean / random_choice, ConstraintCritic.forward (mean / uncertainty / sample),
MLPMultiplier.forward -- HIP vs the CPU oracle on the fixture weights, with the
oracle's live draws replayed. Tolerance (fp32): |d| <= 1e-4 + 1e-4*|ref|."""
import numpy as np
import pytest
import torch

import drpo_amd
from conftest import load_golden
from gpu_helpers import DEV, small_smbpo, close
from oracle import drpo_oracle as O

pytestmark = pytest.mark.gpu


def solver(tag):
    d = load_golden(f'ssac_{tag}')
    alg = small_smbpo(d, str(d['meta/env']))
    sol = alg.solver
    sd0 = {k[4:]: torch.from_numpy(np.array(d[k])) for k in d.files if k.startswith('sd0/')}
    sol.log_alpha.fill_(float(sd0.pop('log_alpha')))
    sol.load_state_dict(sd0, strict=False)
    P = {k: v.detach().cpu() for k, v in sol.state_dict().items()}
    return sol, P


@pytest.mark.parametrize('n', [1, 37, 1000])
def test_policy_act_and_distr(n):
    sol, P = solver('drpo_quad')
    torch.manual_seed(n)
    s = torch.randn(n, sol.state_dim)
    a = sol.act(s.to(DEV), eval=True)
    close(a, O.policy_mean(P, 'actor.net.', s), msg='eval act')
    live = O.LiveRNG()
    a_ref, _, _, _ = O.policy_sample(P, 'actor.net.', s, live)
    tape = drpo_amd.TapeNoise(live.entries)
    a = sol.act(s.to(DEV), eval=False, noise=tape)
    assert tape.done()
    close(a, a_ref, msg='sample act')
    mu, std = O.policy_params(P, 'actor.net.', s)
    dist = sol.actor.distr(s.to(DEV))
    close(dist.base_dist.base_dist.loc, mu, msg='loc')
    close(dist.base_dist.base_dist.scale, std, msg='scale')
    close(dist.mean, torch.tanh(mu), msg='mean')
    # production noise: in range, differs between calls
    a1, a2 = sol.act(s.to(DEV), eval=False), sol.act(s.to(DEV), eval=False)
    assert (a1.abs() <= 1).all() and (n < 8 or not torch.equal(a1, a2))
    # act1 (src/policy.py:16-17)
    close(sol.actor.act1(s[0].to(DEV), eval=True), O.policy_mean(P, 'actor.net.', s[:1])[0], msg='act1')


@pytest.mark.parametrize('tag', ['drpo_quad', 'drpo_point'])
def test_critics_and_multiplier(tag):
    sol, P = solver(tag)
    n = 533
    torch.manual_seed(3)
    s, a = torch.randn(n, sol.state_dim), torch.rand(n, sol.action_dim) * 2 - 1
    sd, ad = s.to(DEV), a.to(DEV)
    ref = O.critic_all(P, 'critic.', s, a)
    got = sol.critic.all(sd, ad)
    for g, r in zip(got, ref):
        close(g, r, msg='q')
    close(sol.critic.min(sd, ad), torch.min(*ref), msg='min')
    close(sol.critic.mean(sd, ad), (ref[0] + ref[1]) / 2, msg='mean')
    tape = drpo_amd.TapeNoise([('choice', np.array(1))])
    close(sol.critic.random_choice(sd, ad, noise=tape), ref[1], msg='random_choice')
    # constraint critic, three modes
    C = sol.con_dim
    close(sol.constraint_critic(sd, ad), O.cons_critic(P, 'constraint_critic.', s, a, 'mean'), msg='cc mean')
    live = O.LiveRNG()
    ub = O.cons_critic(P, 'constraint_critic.', s, a, 'uncertainty', rng=live)
    tape = drpo_amd.TapeNoise(live.entries)
    close(sol.constraint_critic(sd, ad, uncertainty=True, noise=tape), ub, msg='cc uncertainty')
    assert tape.done()
    live = O.LiveRNG()
    m_ref, s_ref, q_ref = O.cons_critic(P, 'constraint_critic.', s, a, 'sample', rng=live)
    tape = drpo_amd.TapeNoise(live.entries)
    m, st, q = sol.constraint_critic(sd, ad, sample=True, noise=tape)
    close(m, m_ref, msg='cc sample mean')
    close(st, s_ref, msg='cc sample std')
    close(q, q_ref, msg='cc sample q')
    assert q.shape == ((n, C) if C > 1 else (n,))
    # multiplier
    qc = O.get_qc(ub, C)
    close(sol.multiplier(sd, qc.to(DEV)), O.multiplier(P, 'multiplier.', s, qc), msg='lam')
    close(sol._get_qc(sol.constraint_critic(sd, ad, uncertainty=True, noise=drpo_amd.TapeNoise(
        [('randn_like', np.zeros((n, C) if C > 1 else n, np.float32))]))), qc, msg='_get_qc')
