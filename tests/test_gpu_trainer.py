"""main.py's loop shape on the HIP trainer vs the reference.

tests/golden/trainer_point-robot.npz was recorded by make_golden.py from the
reference's own SMBPO on point-robot: setup() (uniform-policy collection to
buffer_min + the initial model fit) -> evaluate() -> epoch() (10 real steps,
each with update_models every 4 steps, rollout_and_update, the actor's action
and the uncertainty-shield decision; then log_statistics) -> evaluate() with the
linear shield. Every random draw is replayed from the recorded tape; the env is
tests/pr_env.py (replays the reference's trajectory bit-exactly on the CPU,
tests/test_trainer_host.py).

Tolerances (fp32): real/virtual buffer rows |d| <= 2e-4 + 2e-4|ref| (after 100 SAC
updates, 4 model fits and 10 rollouts the real env is driven by the HIP actor);
parameters |d| <= 2e-3 + 2e-3|ref| (Adam's normalised step amplifies fp32 noise on
near-zero gradients to lr scale over 100 steps); logged statistics rtol 2e-3;
episode lengths, step counts, flags and evaluation lengths exact. The recorded
shield margins (min |qc - threshold| = 1.35 for the step shield, 0.075 for the
evaluation shield) are far above these, so every shield decision is the reference's.
"""
import io
import os

import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu

DEV = torch.device('cuda')
COMP = ('states', 'actions', 'next_states', 'rewards', 'dones', 'violations', 'constraint_values')


def _flag(d, key, default):
    return d[key].item() if key in d.files else default


def _config(d):
    import drpo_amd
    cfg = drpo_amd.SMBPO.Config()
    dist = bool(_flag(d, 'cfg/distributional', True))
    unc = bool(_flag(d, 'cfg/uncertainty', True))
    E, H, B = int(d['meta/E']), int(d['meta/H']), int(d['meta/B'])
    hid, mh = int(d['meta/hidden']), int(d['meta/model_hidden'])
    cfg.update({'horizon': H, 'rollout_batch_size': B, 'buffer_max': int(d['meta/buffer_max']),
                'buffer_min': int(d['cfg/buffer_min']), 'steps_per_epoch': int(d['cfg/steps_per_epoch']),
                'model_update_period': int(d['cfg/model_update_period']),
                'model_initial_steps': int(d['cfg/model_initial_steps']), 'model_steps': int(d['cfg/model_steps']),
                'solver_updates_per_step': 10, 'safe_shield': bool(_flag(d, 'cfg/safe_shield', True)),
                'safe_shield_threshold': float(d['cfg/shield']), 'eval_shield_threshold': float(d['cfg/eval_shield']),
                'eval_shield_type': str(_flag(d, 'cfg/eval_shield_type', 'linear')), 'mode': 'train',
                'model_cfg': {'ensemble_size': E, 'num_elites': int(d['meta/num_elites']), 'hidden_dim': mh,
                              'batch_size': int(d['meta/model_batch']), 'holdout_size': int(d['meta/model_batch'])},
                'sac_cfg': {'batch_size': int(d['meta/sac_batch']), 'hidden_dim': hid,
                            'critic_cfg': {'hidden_dim': hid},
                            'constraint_critic_cfg': {'hidden_dim': hid, 'std_ratio': 2.0},
                            'mlp_multiplier_cfg': {'hidden_dim': hid, 'upper_bound': 50.0},
                            'qc_under_uncertainty': unc, 'distributional_qc': dist, 'target_entropy': -2.0,
                            'penalty_lb': -1.0, 'actor_lr': 1e-4},
                'reward_scale': 2.0, 'alive_bonus': 2.0, 'constraint_offset': 0.5, 'constraint_scale': 10.0})
    return cfg


def _load_sd(alg, d, prefix):
    sd = {k[len(prefix):]: torch.from_numpy(np.array(d[k])) for k in d.files if k.startswith(prefix)}
    la = sd.pop('log_alpha')
    missing, unexpected = alg.load_state_dict(sd, strict=True), None
    alg.solver.log_alpha.fill_(float(la))


def _close(a, b, atol, rtol, msg):
    a = a.detach().cpu().numpy() if torch.is_tensor(a) else np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape, (msg, a.shape, b.shape)
    if a.dtype == bool or b.dtype == bool:
        np.testing.assert_array_equal(a, b, err_msg=msg)
    else:
        np.testing.assert_allclose(a, b, atol=atol, rtol=rtol, err_msg=msg)


# main.py runs: run.sh's DRPO, and run-ablation-1_quadrotor.sh's DRPO-Vanilla (no step
# shield, vanilla certificate, eval_shield_type 'no'), DRPO-Shield-only (vanilla
# certificate, step shield at 0.0, linear evaluation shield) and DRPO-Uncertainty-only
# (no step shield) evaluated with the 'safe' shield
VARIANTS = ['', '_vanilla', '_shield_only', '_uncert_safe']


@pytest.mark.parametrize('variant', VARIANTS)
def test_setup_evaluate_epoch_matches_reference(tmp_path, variant):
    import drpo_amd
    from drpo_amd.checkpoint import CheckpointableData
    from drpo_amd.log import default_log
    from pr_env import PointRobot, TorchEnv
    d = load_golden('trainer_point-robot' + variant)
    default_log.setup(str(tmp_path))
    resets = [np.array(r) for r in d['resets']]
    factory = lambda id=None: TorchEnv(PointRobot(id=id, resets=resets), DEV)  # noqa: E731
    data = CheckpointableData()
    alg = drpo_amd.SMBPO(_config(d), factory, data, 1, device=DEV)
    _load_sd(alg, d, 'sd0/')

    tape = drpo_amd.TapeNoise.from_npz(d, 'setup_tape')
    alg.noise = tape
    alg.setup()
    assert tape.done(), f'setup consumed {tape.pos} of {len(tape.entries)} draws'
    keys = [str(k) for k in d['eval/keys']]
    ev0 = alg.evaluate()
    tape = drpo_amd.TapeNoise.from_npz(d, 'epoch_tape')
    alg.noise = tape
    alg.epoch()
    assert tape.done(), f'epoch consumed {tape.pos} of {len(tape.entries)} draws'
    ev1 = alg.evaluate()
    torch.cuda.synchronize()

    for ev, ref in ((ev0, d['eval/0']), (ev1, d['eval/1'])):
        got = np.array([ev[k] for k in keys])
        for k, g, r in zip(keys, got, ref):
            if 'length' in k:
                assert g == r, (k, g, r)
            else:
                np.testing.assert_allclose(g, r, rtol=2e-3, atol=2e-3, err_msg=k)
    assert len(resets) == 0, 'every recorded training-env reset was used'
    assert int(alg.epochs_completed) == 1
    for name, buf in (('replay', alg.replay_buffer), ('virt', alg.virt_buffer)):
        assert len(buf) == int(d[f'{name}/n']), name
        got = buf.get(as_dict=True)
        for k in COMP:
            _close(got[k], d[f'{name}/{k}'], 2e-4, 2e-4, f'{name}/{k}')
    sd = alg.state_dict()
    for k in d.files:
        if k.startswith('sd1/') and k != 'sd1/log_alpha':
            _close(sd[k[4:]], d[k], 2e-3, 2e-3, k)
    np.testing.assert_allclose(float(alg.solver.log_alpha), float(d['sd1/log_alpha']), rtol=1e-3, atol=1e-4)
    dkeys = [str(k) for k in d['data/keys']]
    assert sorted(data._data) == dkeys
    for i, k in enumerate(dkeys):
        ref = d[f'data/{i:03d}']
        got = np.array([np.nan if v is None else float(v) for v in data[k]], dtype=np.float64)
        assert got.shape == ref.shape, k
        np.testing.assert_allclose(got, ref, rtol=2e-3, atol=2e-3, equal_nan=True, err_msg=k)
    csv_got = open(os.path.join(str(tmp_path), 'episodes.csv')).read().splitlines()
    csv_ref = str(d['episodes_csv']).splitlines()
    assert len(csv_got) == len(csv_ref) and csv_got[:1] == csv_ref[:1]
    for g, r in zip(csv_got[1:], csv_ref[1:]):
        gs, rs = g.split(','), r.split(',')
        for x, y in zip(gs, rs):
            if x in ('True', 'False', '') or y in ('True', 'False', ''):
                assert x == y, (g, r)
            else:
                np.testing.assert_allclose(float(x), float(y), rtol=1e-4, atol=1e-4)


def test_reference_checkpoint_round_trip_on_device(tmp_path):
    """A ckpt written by the reference's Checkpointer loads into the HIP SMBPO, drives a
    rollout, and saves back with the same 103 keys and values (f3)."""
    import drpo_amd
    from drpo_amd.checkpoint import Checkpointer
    from fake_envs import ENVS
    d = load_golden('checkpoint_point-robot')
    ref_sd = torch.load(io.BytesIO(d['ckpt_bytes'].tobytes()), map_location='cpu', weights_only=True)
    cfg = drpo_amd.SMBPO.Config()
    E, hid, mh = int(d['meta/E']), int(d['meta/hidden']), int(d['meta/model_hidden'])
    cfg.update({'horizon': int(d['meta/H']), 'rollout_batch_size': int(d['meta/B']), 'buffer_max': 1000,
                'model_cfg': {'ensemble_size': E, 'num_elites': int(d['meta/num_elites']), 'hidden_dim': mh},
                'sac_cfg': {'hidden_dim': hid, 'critic_cfg': {'hidden_dim': hid},
                            'constraint_critic_cfg': {'hidden_dim': hid}, 'mlp_multiplier_cfg': {'hidden_dim': hid}}})
    alg = drpo_amd.SMBPO(cfg, lambda id=None: ENVS['point-robot'](), None, 1, device=DEV)
    open(tmp_path / 'ckpt_3.pt', 'wb').write(d['ckpt_bytes'].tobytes())
    ck = Checkpointer(alg, tmp_path, 'ckpt_{}.pt')
    assert ck.load_latest([0, 3]) == 3
    assert int(alg.epochs_completed) == 3
    rng = np.random.RandomState(0)
    s0 = torch.from_numpy(rng.uniform(-2, 2, size=(64, alg.state_dim)).astype(np.float32)).to(DEV)
    alg.model_ensemble._elite_inds = [0, 1]
    out = alg.rollout(alg.actor, initial_states=s0)
    assert 0 < len(out) <= 64 * alg.horizon
    ck.save(4)
    back = torch.load(tmp_path / 'ckpt_4.pt', map_location='cpu', weights_only=True)
    assert set(back) == set(ref_sd)
    for k, v in ref_sd.items():
        assert torch.equal(back[k].cpu(), v), k
