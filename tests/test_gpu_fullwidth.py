"""Safe-SAC update at the reference's FULL widths (hidden 256, quadrotor dims, DRPO
flags) against the CPU oracle with its draws replayed. The golden fixtures use
reduced widths (48), so this is the test that covers the 256-wide paths: 16-step
unrolled k-loops, two column blocks per wave, and the multi-job forward's paired
constraint-critic heads (one paired hidden layer + one narrow pair over the trunk
output, mlp.hip heads_pair). Tolerances as tests/test_gpu_sac.py: losses rtol 1e-4,
parameters |d| <= 3e-5 + 1e-4*|ref| after each Adam step."""
import numpy as np
import pytest
import torch

import drpo_amd
from gpu_helpers import DEV
from oracle import drpo_oracle as O

pytestmark = pytest.mark.gpu
PARAM_ATOL, PARAM_RTOL = 3e-5, 1e-4


def _check(sol, P, msg):
    sd = sol.state_dict()
    bad = []
    for k, exp in P.items():
        if k not in sd:
            continue
        got = sd[k].detach().cpu().numpy()
        e = exp.numpy()
        err = np.abs(got - e) - (PARAM_ATOL + PARAM_RTOL * np.abs(e))
        if (err > 0).any():
            bad.append((k, float(np.abs(got - e).max()), int((err > 0).sum()), e.size))
    assert not bad, f'{msg}: {bad[:6]}'


def test_full_width_sac_updates_vs_oracle():
    import bench
    B = 512
    alg = bench.make_alg(DEV, B, 10, 7, 0, bench.QUAD_JSON)
    sol = alg.solver
    sd = {k: v.detach().cpu().clone() for k, v in alg.state_dict().items()}
    Ps = {k[len('solver.'):]: v for k, v in sd.items() if k.startswith('solver.') and
          not k.startswith('solver.model_ensemble') and k != 'solver.total_updates'}
    orc = O.SSACOracle(Ps, dict(batch_size=B, target_entropy=-2.0, penalty_lb=-1.0, actor_lr=1e-4,
                                updates_per_training=sol.updates_per_training), 2, 2)
    rng = np.random.RandomState(4)
    rep = bench.synth_replay('quadrotor', 4000, rng)
    idx = rng.randint(0, 4000, B)
    h = torch.from_numpy(rep['constraint_values'])[idx]
    batch = (torch.from_numpy(rep['states'])[idx], torch.from_numpy(rep['actions'])[idx],
             torch.from_numpy(rep['next_states'])[idx], torch.from_numpy(rep['rewards'])[idx] * 2.0 + 2.0,
             torch.zeros(B, dtype=torch.bool), torch.zeros(B, dtype=torch.bool), h * 10.0 + (h > 0).float() * 0.5)
    dev_batch = [x.to(DEV) for x in batch]

    live = O.LiveRNG()
    lq_ref, lqc_ref = orc.update_critic(*batch, live)
    tape = drpo_amd.TapeNoise(live.entries)
    lq, lqc = sol.update_critic(*dev_batch, noise=tape)
    torch.cuda.synchronize()
    assert tape.done()
    np.testing.assert_allclose(lq.item(), float(lq_ref), rtol=1e-4)
    np.testing.assert_allclose(lqc.item(), float(lqc_ref), rtol=1e-4)
    _check(sol, orc.P, 'after update_critic')

    live = O.LiveRNG()
    orc.update_actor_and_alpha(batch[0], live)
    tape = drpo_amd.TapeNoise(live.entries)
    sol.update_actor_and_alpha(dev_batch[0], noise=tape)
    torch.cuda.synchronize()
    assert tape.done()
    np.testing.assert_allclose(sol.log_alpha.item(), float(orc.log_alpha), rtol=1e-5, atol=1e-6)
    _check(sol, orc.P, 'after update_actor_and_alpha')

    live = O.LiveRNG()
    orc.update_multiplier(batch[0], live)
    tape = drpo_amd.TapeNoise(live.entries)
    sol.update_multiplier(dev_batch[0], noise=tape)
    torch.cuda.synchronize()
    assert tape.done()
    _check(sol, orc.P, 'after update_multiplier')
