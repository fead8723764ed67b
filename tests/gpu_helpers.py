"""Shared helpers for the GPU parity tests."""
import numpy as np
import torch

import drpo_amd
from fake_envs import ENVS
from oracle import drpo_oracle as O

DEV = torch.device('cuda')
COMP = O.COMPONENTS


def small_smbpo(d, env, factory=None):
    cfg = drpo_amd.SMBPO.Config()
    E, H, B = int(d['meta/E']), int(d['meta/H']), int(d['meta/B'])
    hid, mh = int(d['meta/hidden']), int(d['meta/model_hidden'])
    cfg.update({'horizon': H, 'rollout_batch_size': B, 'buffer_max': int(d['meta/buffer_max']),
                'steps_per_epoch': 2, 'solver_updates_per_step': 10,
                'model_cfg': {'ensemble_size': E, 'num_elites': int(d['meta/num_elites']), 'hidden_dim': mh,
                              'batch_size': int(d['meta/model_batch']), 'holdout_size': int(d['meta/model_batch'])},
                'sac_cfg': {'batch_size': int(d['meta/sac_batch']), 'hidden_dim': hid,
                            'critic_cfg': {'hidden_dim': hid}, 'constraint_critic_cfg': {'hidden_dim': hid},
                            'mlp_multiplier_cfg': {'hidden_dim': hid},
                            'qc_under_uncertainty': bool(d['meta/uncertainty']),
                            'distributional_qc': bool(d['meta/distributional']), 'target_entropy': -2.0,
                            'penalty_lb': -1.0, 'actor_lr': 1e-4},
                'reward_scale': 2.0, 'alive_bonus': 2.0, 'constraint_offset': 0.5, 'constraint_scale': 10.0})
    flags = {k[len('flag/'):]: d[k].item() for k in d.files if k.startswith('flag/')}
    if flags:                          # solver-flag fixtures (make_golden.SOLVER_FLAG_CASES)
        cfg.update({'sac_cfg': flags})
    return drpo_amd.SMBPO(cfg, factory or (lambda id=None: ENVS[env]()), None, 1, device=DEV)


def load_sd(alg, d, prefix):
    sd = {k[len(prefix):]: torch.from_numpy(np.array(d[k])) for k in d.files if k.startswith(prefix)}
    sd.pop('log_alpha', None)
    missing, unexpected = alg.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected


def fill_replay(alg, d):
    rows = {k: torch.from_numpy(d['replay/' + k]).to(DEV) for k in COMP}
    half = len(rows['states']) // 2
    alg.replay_buffer.extend(**{k: v[:half] for k, v in rows.items()})
    alg.replay_buffer.extend(**{k: v[half:] for k, v in rows.items()})


def close(a, b, tol=1e-4, msg=''):
    a = a.detach().cpu().numpy() if torch.is_tensor(a) else np.asarray(a)
    b = b.detach().cpu().numpy() if torch.is_tensor(b) else np.asarray(b)
    assert a.shape == b.shape, (msg, a.shape, b.shape)
    if a.dtype == bool or b.dtype == bool:
        np.testing.assert_array_equal(a, b, err_msg=msg)
    else:
        np.testing.assert_allclose(a, b, rtol=tol, atol=tol, err_msg=msg)


