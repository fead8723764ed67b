"""HIP safe-SAC update parity against the reference's golden fixtures (recorded
noise). Tolerances (fp32, after Adam steps): losses rtol 1e-4; parameters
|d| <= 3e-5 + 1e-4*|ref| (one Adam step moves a weight by ~lr = 3e-4, so this
catches any wrong gradient sign/magnitude while allowing fp32 summation-order
differences); log_alpha likewise."""
import numpy as np
import pytest
import torch

import drpo_amd
from conftest import load_golden
from gpu_helpers import DEV, COMP, small_smbpo, load_sd, close

pytestmark = pytest.mark.gpu
PARAM_ATOL, PARAM_RTOL = 3e-5, 1e-4


def solver_sd(d, prefix):
    return {k[len(prefix):]: torch.from_numpy(np.array(d[k])) for k in d.files if k.startswith(prefix)}


def check_params(module, ref, msg, skip=('model_ensemble', 'total_updates', 'log_alpha')):
    sd = module.state_dict()
    bad = []
    for k, v in ref.items():
        if k.startswith(skip):
            continue
        got = sd[k].detach().cpu().numpy()
        exp = v.numpy()
        err = np.abs(got - exp) - (PARAM_ATOL + PARAM_RTOL * np.abs(exp))
        if (err > 0).any():
            bad.append((k, float(np.abs(got - exp).max()), int((err > 0).sum()), exp.size))
    assert not bad, f'{msg}: {bad[:6]}'


@pytest.mark.parametrize('tag', ['drpo_point', 'drpo_quad', 'vanilla_quad', 'robust_quad', 'robust_point',
                                 'scalar_mult_point', 'scalar_mult_quad', 'fixed_alpha_quad', 'log_alpha_point',
                                 'cost_point', 'cost_quad', 'fullwidth_quad'])
def test_ssac_updates_match_reference(tag):
    """scalar_mult..log_alpha are the SSAC configuration branches (scalar softplus
    multiplier with clamp(Qc) in the actor loss, autotune_alpha=False,
    use_log_alpha_loss=True); cost_* the constrained_fcn='cost' certificate (one-step
    violation cost target from the actor's next action, no safe-actor update);
    fullwidth_quad the reference's default widths (every net 256 wide: the production
    pair / chain / paired-heads tilings), B = 64."""
    d = load_golden(f'ssac_{tag}')
    env = str(d['meta/env'])
    alg = small_smbpo(d, env)
    sol = alg.solver
    sd0 = solver_sd(d, 'sd0/')
    sol.log_alpha.fill_(float(sd0.pop('log_alpha')))
    missing, unexpected = sol.load_state_dict(sd0, strict=False)
    assert not unexpected
    if 'model/elite_inds' in d.files:     # robust branch samples the dynamics model
        alg.model_ensemble._elite_inds = list(d['model/elite_inds'])
    batch = [torch.from_numpy(d['in/' + k]).to(DEV) for k in ['s', 'a', 's2', 'r', 'd', 'v', 'h']]
    tape = drpo_amd.TapeNoise.from_npz(d, 'critic_tape')
    lq, lqc = sol.update_critic(*batch, noise=tape)
    torch.cuda.synchronize()
    assert tape.done()
    np.testing.assert_allclose(lq.item(), float(d['out/lq']), rtol=1e-4)
    np.testing.assert_allclose(lqc.item(), float(d['out/lqc']), rtol=1e-4)
    check_params(sol, solver_sd(d, 'sd1/'), 'after update_critic')

    tape = drpo_amd.TapeNoise.from_npz(d, 'actor_tape')
    sol.update_actor_and_alpha(batch[0], noise=tape)
    torch.cuda.synchronize()
    assert tape.done()
    ref2 = solver_sd(d, 'sd2/')
    np.testing.assert_allclose(sol.log_alpha.item(), float(ref2['log_alpha']), rtol=1e-5, atol=1e-6)
    check_params(sol, ref2, 'after update_actor_and_alpha')

    tape = drpo_amd.TapeNoise.from_npz(d, 'mult_tape')
    sol.update_multiplier(batch[0], noise=tape)
    torch.cuda.synchronize()
    assert tape.done()
    check_params(sol, solver_sd(d, 'sd3/'), 'after update_multiplier')
    lrs = [sol.critic_optimizer.lr, sol.actor_optimizer.lr, sol.actor_safe_optimizer.lr, sol.multiplier_optimizer.lr]
    np.testing.assert_array_equal(np.array(lrs), d['lr3'])


@pytest.mark.parametrize('tag', ['point-robot', 'quadrotor', 'cost_point'])
def test_rollout_and_update_matches_reference(tag):
    """Two full SMBPO.rollout_and_update() calls (rollout + 10 update_solver each, the
    reference cadence) from the post-fit state of the fixture. cost_point: the
    constrained_fcn='cost' certificate through the device batch path (violation flags
    gathered from the buffers)."""
    d = load_golden(f'smbpo_update_{tag}')
    env = str(d['meta/env'])
    alg = small_smbpo(d, env)
    sd1 = {k[len('sd1/'):]: torch.from_numpy(np.array(d[k])) for k in d.files if k.startswith('sd1/')}
    la = sd1.pop('log_alpha', None)
    alg.load_state_dict(sd1, strict=False)
    alg.solver.log_alpha.fill_(float(d['sd0/log_alpha']) if la is None else float(la))
    rows = {k: torch.from_numpy(d['replay/' + k]).to(DEV) for k in COMP}
    half = len(rows['states']) // 2
    alg.replay_buffer.extend(**{k: v[:half] for k, v in rows.items()})
    alg.replay_buffer.extend(**{k: v[half:] for k, v in rows.items()})
    alg.model_ensemble._elite_inds = list(d['fit/elite_inds'])
    for r in range(2):
        tape = drpo_amd.TapeNoise.from_npz(d, f'rau{r}_tape')
        alg.rollout_and_update(noise=tape)
        torch.cuda.synchronize()
        assert tape.done()
    assert len(alg.virt_buffer) == int(d['virt/n'])
    got = alg.virt_buffer.get(as_dict=True)
    for k in COMP:
        close(got[k], d['virt/' + k], tol=1e-3, msg=k)
    ref = {k[len('sd2/'):]: torch.from_numpy(np.array(d[k])) for k in d.files if k.startswith('sd2/')}
    np.testing.assert_allclose(alg.solver.log_alpha.item(), float(ref.pop('log_alpha')), rtol=1e-4, atol=1e-6)
    check_params(alg, ref, 'after 2x rollout_and_update',
                 skip=('model_ensemble', 'solver.model_ensemble', 'solver.total_updates', 'episodes', 'steps',
                       'n_viol', 'epochs'))
    lq = np.array([x.item() for x in alg.recent_critic_losses])
    np.testing.assert_allclose(lq, d['losses/critic'], rtol=1e-3, atol=1e-5)


def test_actor_arena_rebuild_matches_presized_engine():
    """The actor exchange arena (actor | safe actor grads | alpha-loss partials) is
    rebuilt when a batch larger than it was sized for arrives: the gradients are
    re-homed, the Parameters' .grad views follow, and every cached descriptor is
    dropped. Actor updates at B = 64, 5000 (forces the rebuild), 64 must give bitwise
    the parameters of an engine whose arena was sized for 8192 rows up front."""
    from drpo_amd.rng import DeviceNoise
    d = load_golden('ssac_drpo_quad')
    env = str(d['meta/env'])

    def run(presize):
        alg = small_smbpo(d, env)
        sol = alg.solver
        sd0 = solver_sd(d, 'sd0/')
        sol.log_alpha.fill_(float(sd0.pop('log_alpha')))
        sol.load_state_dict(sd0, strict=False)
        eng = sol.engine
        first = eng.actor_xchg
        if presize:
            eng._actor_arena(presize)
        g = torch.Generator().manual_seed(3)
        noise = DeviceNoise(7)
        for B in (64, 5000, 64):
            obs = torch.randn(B, alg.state_dim, generator=g).to(DEV)
            sol.update_actor_and_alpha(obs, noise=noise)
        torch.cuda.synchronize()
        arena = eng.actor_xchg
        lo, hi = arena.data_ptr(), arena.data_ptr() + 4 * arena.numel()
        for p in list(sol.actor.parameters()) + list(sol.actor_safe.parameters()):
            assert p.grad is not None and lo <= p.grad.data_ptr() < hi, 'a .grad view left on the old arena'
        rebuilt = arena is not first
        return {k: v.detach().clone() for k, v in sol.state_dict().items()}, rebuilt

    a, rebuilt_a = run(None)
    b, _ = run(8192)
    assert rebuilt_a, 'B = 5000 must outgrow the arena sized for the solver batch'
    for k in a:
        assert torch.equal(a[k], b[k]), k



@pytest.mark.parametrize('tag', ['drpo_quad', 'cost_point'])
def test_early_actor_forward_matches_standalone_launch(tag):
    """Production noise: the actor update's first forward rides in the critic update's
    forward launch ('c.f+a', SACEngine._early_actor). Its outputs (actions, log-probs,
    pre-tanh samples and noise, tanh(mu_safe), every saved activation) must be bitwise
    those of the stand-alone 'a.f1' launch at the same Philox counter, and the critic
    update must be unchanged by the extra job."""
    from drpo_amd.rng import DeviceNoise
    d = load_golden(f'ssac_{tag}')
    env = str(d['meta/env'])
    batch = [torch.from_numpy(d['in/' + k]).to(DEV) for k in ['s', 'a', 's2', 'r', 'd', 'v', 'h']]

    def run(early):
        alg = small_smbpo(d, env)
        sol = alg.solver
        sd0 = solver_sd(d, 'sd0/')
        sol.log_alpha.fill_(float(sd0.pop('log_alpha')))
        sol.load_state_dict(sd0, strict=False)
        eng = sol.engine
        orig = eng._critic_step
        eng._critic_step = lambda nz: orig(nz, early_actor=early)
        noise = DeviceNoise(11)
        lq, lqc = sol.update_critic(*batch, noise=noise)
        torch.cuda.synchronize()
        return sol, eng, noise.ctr, (lq.item(), lqc.item())

    sol, eng, ctr, losses = run(True)
    names = ['a.a', 'a.lp', 'a.u', 'a.e', 'a.am', 'a.x'] + ([] if eng.cost else ['a.as', 'a.us', 'a.es'])
    nets = [eng.nets['actor']] + ([] if eng.cost else [eng.nets['safe']])
    early = [eng.ws[k].clone() for k in names] + [y.clone() for n in nets for y in n.sy if y is not None]
    for t in [eng.ws[k] for k in names] + [y for n in nets for y in n.sy if y is not None]:
        t.fill_(float('nan'))
    eng._run_multi('a.f1.test', lambda: eng._actor_f1_jobs(None, None), ctr)
    torch.cuda.synchronize()
    alone = [eng.ws[k] for k in names] + [y for n in nets for y in n.sy if y is not None]
    for i, (x, y) in enumerate(zip(early, alone)):
        assert torch.equal(x, y), f'output {i} differs'
    sol2, _, _, losses2 = run(False)
    assert losses == losses2
    ref = sol2.state_dict()
    for k, v in sol.state_dict().items():
        assert torch.equal(v, ref[k]), k
