"""CPU checks of the trainer-side host pieces (no GPU):

* the test-side point-robot env (tests/pr_env.py) replays the reference's real-env
  trajectory recorded in tests/golden/trainer_point-robot.npz bit-exactly, so the
  GPU trainer test drives the same environment the reference drove;
* the reference's own Checkpointer output (ckpt_3.pt, data.pt bytes in
  tests/golden/checkpoint_point-robot.npz) loads with the safe loader and has the
  key set the build's SMBPO produces (103 keys; duplicate solver.model_ensemble.*;
  no log_alpha);
* DeviceNoise: per-rank device keys differ, host choices agree across ranks.
"""
import io

import numpy as np
import pytest
import torch

from conftest import load_golden
from pr_env import PointRobot


@pytest.mark.parametrize('variant', ['', '_vanilla', '_shield_only', '_uncert_safe'])
def test_pr_env_replays_reference_trajectory(variant):
    d = load_golden('trainer_point-robot' + variant)
    resets = list(d['resets'])
    env = PointRobot(resets=resets)
    S = d['replay/states']
    A = d['replay/actions']
    n = int(d['replay/n'])
    obs = env.reset()
    for t in range(n):
        np.testing.assert_array_equal(obs, S[t], err_msg=f'state {t}')
        obs2, r, done, info = env.step(A[t])
        np.testing.assert_array_equal(obs2, d['replay/next_states'][t], err_msg=f'next state {t}')
        assert np.float32(r) == d['replay/rewards'][t], t
        assert done == bool(d['replay/dones'][t]), t
        assert info['violation'] == bool(d['replay/violations'][t]), t
        assert np.float32(info['constraint_value']) == d['replay/constraint_values'][t], t
        np.testing.assert_array_equal(env.check_done(obs2), done)
        if done:
            obs = env.reset()
        else:
            obs = obs2
    assert not resets or len(resets) <= 1


def test_reference_checkpoint_loads_safely_with_build_keys():
    d = load_golden('checkpoint_point-robot')
    sd = torch.load(io.BytesIO(d['ckpt_bytes'].tobytes()), map_location='cpu', weights_only=True)
    data = torch.load(io.BytesIO(d['data_bytes'].tobytes()), map_location='cpu', weights_only=True)
    assert len(sd) == 103
    assert 'solver.log_alpha' not in sd and not any(k.endswith('log_alpha') for k in sd)
    dup = [k for k in sd if k.startswith('solver.model_ensemble.')]
    assert dup and all(torch.equal(sd[k], sd['model_ensemble.' + k[len('solver.model_ensemble.'):]]) for k in dup)
    assert int(sd['epochs_completed']) == 3
    assert set(data) == {'critic loss', 'eval return mean'}
    for k in d.files:
        if k.startswith('sd/'):
            np.testing.assert_array_equal(sd[k[3:]].numpy(), d[k])


def test_build_state_dict_matches_reference_checkpoint_keys():
    import drpo_amd
    from fake_envs import ENVS
    d = load_golden('checkpoint_point-robot')
    sd = torch.load(io.BytesIO(d['ckpt_bytes'].tobytes()), map_location='cpu', weights_only=True)
    cfg = drpo_amd.SMBPO.Config()
    E, hid, mh = int(d['meta/E']), int(d['meta/hidden']), int(d['meta/model_hidden'])
    cfg.update({'model_cfg': {'ensemble_size': E, 'num_elites': int(d['meta/num_elites']), 'hidden_dim': mh},
                'sac_cfg': {'hidden_dim': hid, 'critic_cfg': {'hidden_dim': hid},
                            'constraint_critic_cfg': {'hidden_dim': hid}, 'mlp_multiplier_cfg': {'hidden_dim': hid}},
                'buffer_max': 1000})
    alg = drpo_amd.SMBPO(cfg, lambda id=None: ENVS['point-robot'](), None, 1, device=torch.device('cpu'))
    ours = alg.state_dict()
    assert set(ours) == set(sd)
    for k in sd:
        assert tuple(ours[k].shape) == tuple(sd[k].shape), k
        assert ours[k].dtype == sd[k].dtype, k
    alg.load_state_dict(sd)
    for k in sd:
        assert torch.equal(alg.state_dict()[k].cpu(), sd[k]), k


def test_device_noise_rank_keys_and_shared_host_choices():
    from drpo_amd.rng import DeviceNoise
    a, b = DeviceNoise(7, rank=0), DeviceNoise(7, rank=1)
    assert a.seed == 7 and b.seed != a.seed
    assert [a.choice(5) for _ in range(50)] == [b.choice(5) for _ in range(50)]
    c = DeviceNoise(8, rank=0)
    assert [DeviceNoise(7, rank=0).choice(5) for _ in range(1)] is not None
    assert [c.choice(1000) for _ in range(20)] != [DeviceNoise(7, rank=0).choice(1000) for _ in range(20)]
    torch.manual_seed(1234)
    assert DeviceNoise(None, rank=0).seed == 1234


def test_checkpointer_round_trip(tmp_path):
    from drpo_amd.checkpoint import CheckpointableData, Checkpointer
    data = CheckpointableData()
    data.append('x', 1.5)
    data.append('x', None)
    Checkpointer(data, tmp_path, 'data.pt').save()
    d2 = CheckpointableData()
    assert Checkpointer(d2, tmp_path, 'data.pt').try_load()
    assert d2['x'] == [1.5, None]
    assert Checkpointer(d2, tmp_path, 'ckpt_{}.pt').load_latest([0, 20]) is None
