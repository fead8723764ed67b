"""Generate the golden fixtures under tests/golden/*.npz by running the REFERENCE.

Runs ONLY in the build container (it imports /root/reference, which does not
exist on the GPU box). Usage:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

The reference runs unmodified (CPU, torch.set_num_threads(4) as src/cli.py:108);
tests/golden/tape.py records every random draw in call order so the build can
replay them. Widths are reduced (the reference Config classes allow it) and
deliberately NOT multiples of 16 so the HIP kernels' padding paths are covered;
full widths are covered by HIP-vs-oracle tests at the BASELINE configs.

Environments: point-robot and tracking use the reference env classes directly
(src/env/point_robot.py, src/env/tracking/pyth_veh3dofconti_surrcstr_data.py).
Quadrotor and cartpole need safe_control_gym / mujoco (absent), so their
batched constraint functions are driven here through the reference's own
BoundedConstraint (src/env/poles/constraints.py:216-247) with the bounds from
src/env/quadrotor/constrained_tracking_reset.yaml and
src/env/poles/inverted_pendulum.py:16-34. The quadrotor out-of-bound
thresholds (x_threshold, z_threshold) live in safe_control_gym: PARITY UNPINNED
(we use 2.0 / 3.0, documented in DESIGN.md).
"""
import copy
import hashlib
import math
import os
import random
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = '/root/reference'
sys.path.insert(0, os.path.join(HERE, '_stubs'))
sys.path.insert(0, REF)
sys.path.insert(0, HERE)
os.environ.setdefault('PYTHONDONTWRITEBYTECODE', '1')

import torch  # noqa: E402

torch.set_num_threads(4)

from tape import Tape  # noqa: E402
import gym  # noqa: E402  (stub)
from src.log import default_log  # noqa: E402
from src.smbpo import SMBPO  # noqa: E402
from src.env.point_robot import PointRobot  # noqa: E402
from src.env.tracking.pyth_veh3dofconti_surrcstr_data import SimuVeh3dofcontiSurrCstr  # noqa: E402
from src.env.poles.constraints import BoundedConstraint, ConstrainedVariableType  # noqa: E402
from src.env.torch_wrapper import TorchWrapper  # noqa: E402
from src.checkpoint import CheckpointableData  # noqa: E402
from src.util import set_seed  # noqa: E402

QUAD_X_THRESHOLD = 2.0   # safe_control_gym value: unpinned here
QUAD_Z_THRESHOLD = 3.0


class FakeQuadrotor(gym.Env):
    """Quadrotor observation/constraint surface of src/env/quadrotor/quadrotor.py:35-158
    without the safe_control_gym simulator (obs 12, act 2, con_dim 2)."""

    def __init__(self, id=None):
        self.observation_space = gym.spaces.Box(-np.inf, np.inf, shape=(12,))
        self.action_space = gym.spaces.Box(-1.0, 1.0, shape=(2,))
        self.constraints = BoundedConstraint(12, lower_bounds=[0.5], upper_bounds=[1.5],
                                             constrained_variable=ConstrainedVariableType.STATE,
                                             active_dims=[2])
        self.con_dim = 2
        self._max_episode_steps = 360
        self.x_threshold, self.z_threshold = QUAD_X_THRESHOLD, QUAD_Z_THRESHOLD

    def check_done(self, states):
        if len(states.shape) == 1:
            states = states[np.newaxis, ...]
        th = 85 * math.pi / 180
        x, z, theta = states[..., 0], states[..., 2], states[..., 4]
        done = (x < -self.x_threshold) + (x > self.x_threshold) + (z < -self.z_threshold) + \
            (z > self.z_threshold) + (theta < -th) + (theta > th)
        return np.logical_or(done, self.check_violation(states))

    def check_violation(self, states):
        if len(states.shape) == 1:
            states = states[np.newaxis, ...]
        return self.constraints.is_violated(states)

    def get_constraint_values(self, states):
        if len(states.shape) == 1:
            states = states[np.newaxis, ...]
        return np.squeeze(self.constraints.get_value(states))


class FakeCartpole(gym.Env):
    """Constraint surface of src/env/poles/inverted_pendulum.py:9-121 (obs 4, act 1, con 4)."""

    def __init__(self, id=None):
        self.observation_space = gym.spaces.Box(-np.inf, np.inf, shape=(4,))
        self.action_space = gym.spaces.Box(-1.0, 1.0, shape=(1,))
        self.constraints = BoundedConstraint(4, lower_bounds=[-0.9, -0.2], upper_bounds=[0.9, 0.2],
                                             constrained_variable=ConstrainedVariableType.STATE,
                                             active_dims=[0, 1])
        self.con_dim = 4
        self._max_episode_steps = 1000

    def check_done(self, states):
        return self.constraints.is_violated(states)

    def check_violation(self, states):
        return self.constraints.is_violated(states)

    def get_constraint_values(self, states):
        if len(states.shape) == 1:
            states = states[np.newaxis, ...]
        return np.squeeze(self.constraints.get_value(states))


def env_factory_for(name):
    if name == 'point-robot':
        return lambda id=None: TorchWrapper(PointRobot(id=id))
    if name == 'quadrotor':
        return lambda id=None: TorchWrapper(FakeQuadrotor(id=id))
    if name == 'cartpole':
        return lambda id=None: TorchWrapper(FakeCartpole(id=id))
    if name == 'tracking':
        return lambda id=None: TorchWrapper(SimuVeh3dofcontiSurrCstr(ref_num=1, surr_veh_num=1))
    raise KeyError(name)


def t2n(x):
    return x.detach().cpu().numpy().copy()


def sd_dict(module, prefix='sd/'):
    return {prefix + k: t2n(v) for k, v in module.state_dict().items()}


def synth_states(name, n, rng):
    """Synthetic states per SURVEY.md §8(d)."""
    if name == 'quadrotor':
        s = rng.normal(0, 0.1, size=(n, 12))
        s[:, 0] = rng.uniform(-1, 1, n)
        s[:, 2] = rng.uniform(0.8, 1.2, n)
        s[:, 4] = rng.uniform(-0.1, 0.1, n)
    elif name == 'point-robot':
        s = np.zeros((n, 11))
        xy = rng.uniform(-2.5, 2.5, size=(n, 2))
        v = rng.uniform(0.5, 2.0, n)
        th = rng.uniform(np.pi / 4, 3 * np.pi / 4, n)
        s[:, 0:2] = xy
        s[:, 2] = v
        s[:, 3] = np.cos(th)
        s[:, 4] = np.sin(th)
        s[:, 5:] = rng.normal(0, 1, size=(n, 6))
    elif name == 'cartpole':
        s = rng.normal(0, 0.1, size=(n, 4))
        s[:, 0] = rng.uniform(-0.5, 0.5, n)
        s[:, 1] = rng.uniform(-0.1, 0.1, n)
    elif name == 'tracking':
        s = rng.normal(0, 0.5, size=(n, 51))
        s[:, 0] = rng.uniform(-2, 2, n)
        s[:, 1] = rng.uniform(-1, 1, n)
        s[:, 2] = rng.uniform(-0.5, 0.5, n)
        s[:, 47] = rng.uniform(-12, 12, n)
        s[:, 48] = rng.uniform(-4, 4, n)
        s[:, 49] = rng.normal(0, 0.2, n)
    else:
        raise KeyError(name)
    return s.astype(np.float32)


def fill_replay(alg, name, n, seed, con_dim):
    rng = np.random.RandomState(seed)
    s = synth_states(name, n, rng)
    a = rng.uniform(-1, 1, size=(n, alg.action_dim)).astype(np.float32)
    s2 = (s + rng.normal(0, 1e-3, size=s.shape)).astype(np.float32)
    r = rng.normal(0, 1, n).astype(np.float32)
    env = alg.real_env
    h = env.get_constraint_values(s2).astype(np.float32)
    d = np.asarray(env.check_done(s2)).astype(bool)
    v = np.asarray(env.check_violation(s2)).astype(bool)
    data = dict(states=s, actions=a, next_states=s2, rewards=r, dones=d, violations=v, constraint_values=h)
    data = {k: torch.from_numpy(np.ascontiguousarray(x)) for k, x in data.items()}
    # two extends so the circular buffer wraps when n > capacity
    half = n // 2
    alg.replay_buffer.extend(**{k: x[:half] for k, x in data.items()})
    alg.replay_buffer.extend(**{k: x[half:] for k, x in data.items()})
    return {'replay/' + k: x.numpy() for k, x in data.items()}


def small_config(name, B=64, H=5, E=4, elites=3, model_hidden=40, hidden=48,
                 distributional=True, uncertainty=True, buffer_max=1000, sac_batch=32):
    cfg = copy.deepcopy(SMBPO.Config())
    upd = {
        'horizon': H, 'rollout_batch_size': B, 'buffer_max': buffer_max, 'buffer_min': 10,
        'steps_per_epoch': 2, 'solver_updates_per_step': 10,
        'model_cfg': {'ensemble_size': E, 'num_elites': elites, 'hidden_dim': model_hidden,
                      'batch_size': 64, 'holdout_size': 64},
        'sac_cfg': {'batch_size': sac_batch, 'hidden_dim': hidden,
                    'critic_cfg': {'hidden_dim': hidden},
                    'constraint_critic_cfg': {'hidden_dim': hidden, 'std_ratio': 2.0},
                    'mlp_multiplier_cfg': {'hidden_dim': hidden, 'upper_bound': 50.0},
                    'qc_under_uncertainty': uncertainty, 'distributional_qc': distributional,
                    'target_entropy': -2.0, 'penalty_lb': -1.0, 'actor_lr': 1e-4},
        'reward_scale': 2.0, 'alive_bonus': 2.0, 'constraint_offset': 0.5, 'constraint_scale': 10.0,
    }
    cfg.update(upd)
    return cfg


def build_alg(name, cfg, seed, epochs=1):
    set_seed(seed)
    alg = SMBPO(cfg, env_factory_for(name), CheckpointableData(), epochs)
    return alg


def meta(name, cfg, alg):
    m = cfg.model_cfg
    s = cfg.sac_cfg
    return {
        'meta/env': np.array(name), 'meta/S': np.array(alg.state_dim), 'meta/A': np.array(alg.action_dim),
        'meta/C': np.array(alg.con_dim), 'meta/E': np.array(m.ensemble_size),
        'meta/num_elites': np.array(m.num_elites), 'meta/model_hidden': np.array(m.hidden_dim),
        'meta/hidden': np.array(s.hidden_dim), 'meta/B': np.array(cfg.rollout_batch_size),
        'meta/H': np.array(cfg.horizon), 'meta/buffer_max': np.array(cfg.buffer_max),
        'meta/sac_batch': np.array(s.batch_size), 'meta/distributional': np.array(s.distributional_qc),
        'meta/uncertainty': np.array(s.qc_under_uncertainty),
        'meta/model_batch': np.array(m.batch_size),
    }


def gen_constraints(out):
    rng = np.random.RandomState(7)
    d = {}
    for name in ['point-robot', 'quadrotor', 'cartpole', 'tracking']:
        env = env_factory_for(name)().env
        s = synth_states(name, 257, rng)
        # widen the spread so every branch fires
        s = s * np.float32(1.8)
        if name == 'point-robot':
            s[:8, 0:2] = [[3.0, 0.0], [3.0000002, 0.0], [-3.0, 1.0], [0.0, -3.0000002],
                          [2.2, 2.5], [2.2, 2.5000002], [0.4, -0.4], [-0.4, 0.4]]
        if name == 'quadrotor':
            s[:6, 2] = [0.5, 1.5, 0.49999997, 1.5000001, 0.0, 3.5]
        if name == 'cartpole':
            s[:4, 0] = [0.9, -0.9, 0.90000004, -0.90000004]
        d[f'{name}/states'] = s
        d[f'{name}/done'] = np.asarray(env.check_done(s)).astype(bool)
        d[f'{name}/violation'] = np.asarray(env.check_violation(s)).astype(bool)
        d[f'{name}/h'] = np.asarray(env.get_constraint_values(s), dtype=np.float64)
    np.savez_compressed(os.path.join(out, 'constraints.npz'), **d)


def gen_rollout(out, name, seed, cfg=None, tag=None, keep=None):
    """keep: state-dict key prefixes stored (None: all)."""
    cfg = cfg or small_config(name)
    alg = build_alg(name, cfg, seed)
    d = meta(name, cfg, alg)
    d.update({k: v for k, v in sd_dict(alg).items() if keep is None or k[3:].startswith(keep)})
    d.update(fill_replay(alg, name, 1200, seed + 1, alg.con_dim))
    states = alg.replay_buffer.get('states')
    alg.model_ensemble.state_normalizer.fit(states)
    alg.model_ensemble._elite_inds = [2, 0, 3]
    d['model/elite_inds'] = np.array(alg.model_ensemble._elite_inds)
    d['model/norm_mean'] = t2n(alg.model_ensemble.state_normalizer.mean)
    d['model/norm_std'] = t2n(alg.model_ensemble.state_normalizer.std)
    with Tape() as tp:
        buf = alg.rollout(alg.actor)
    d.update(tp.to_npz_dict('tape'))
    n = len(buf)
    d['out/n'] = np.array(n)
    for k, v in alg.virt_buffer.get(as_dict=True).items():
        d['out/' + k] = t2n(v)
    np.savez_compressed(os.path.join(out, f'rollout_{tag or name}.npz'), **d)


def gen_ensemble(out, name, seed):
    cfg = small_config(name)
    alg = build_alg(name, cfg, seed)
    model = alg.model_ensemble
    d = meta(name, cfg, alg)
    d.update(sd_dict(model, 'sd/'))
    d.update(fill_replay(alg, name, 1200, seed + 1, alg.con_dim))
    rng = np.random.RandomState(seed + 2)
    s = torch.from_numpy(synth_states(name, 37, rng))
    a = torch.from_numpy(rng.uniform(-1, 1, size=(37, alg.action_dim)).astype(np.float32))
    model.state_normalizer.fit(alg.replay_buffer.get('states'))
    d['model/norm_mean'] = t2n(model.state_normalizer.mean)
    d['model/norm_std'] = t2n(model.state_normalizer.std)
    d['in/s'], d['in/a'] = s.numpy(), a.numpy()
    with torch.no_grad():
        mu, lv = model._forward1(s, a, 1)
    d['out/f1_mean'], d['out/f1_logvar'] = t2n(mu), t2n(lv)
    model._elite_inds = [1, 3]
    with Tape() as tp, torch.no_grad():
        s2, r = model.sample(s, a)
    d.update(tp.to_npz_dict('sample_tape'))
    d['out/sample_s2'], d['out/sample_r'] = t2n(s2), t2n(r)
    E = cfg.model_cfg.ensemble_size
    se = torch.from_numpy(synth_states(name, E * 11, rng)).reshape(E, 11, -1)
    ae = torch.from_numpy(rng.uniform(-1, 1, size=(E, 11, alg.action_dim)).astype(np.float32))
    with torch.no_grad():
        mu_all, lv_all = model._forward_all(se, ae)
    d['in/se'], d['in/ae'] = se.numpy(), ae.numpy()
    d['out/fall_mean'], d['out/fall_logvar'] = t2n(mu_all), t2n(lv_all)
    # compute_loss value and gradients (ragged: 4E+3 rows are truncated to 4E)
    nl = 4 * E + 3
    sl = torch.from_numpy(synth_states(name, nl, rng))
    al = torch.from_numpy(rng.uniform(-1, 1, size=(nl, alg.action_dim)).astype(np.float32))
    tl = torch.from_numpy(np.concatenate([synth_states(name, nl, rng), rng.normal(0, 1, (nl, 1))], 1).astype(np.float32))
    model.optimizer.zero_grad()
    loss = model.compute_loss(sl, al, tl)
    loss.backward()
    d['in/loss_s'], d['in/loss_a'], d['in/loss_t'] = sl.numpy(), al.numpy(), tl.numpy()
    d['out/loss'] = t2n(loss)
    for k, p in model.named_parameters():
        d['grad/' + k] = t2n(p.grad)
    model.optimizer.zero_grad()
    # fit(steps=3) from the replay buffer
    with Tape() as tp:
        losses = model.fit(alg.replay_buffer, steps=3)
    d.update(tp.to_npz_dict('fit_tape'))
    d['out/fit_losses'] = np.array(losses, dtype=np.float64)
    d['out/elite_inds'] = np.array(model._elite_inds)
    d.update(sd_dict(model, 'fit_sd/'))
    np.savez_compressed(os.path.join(out, f'ensemble_{name}.npz'), **d)


def synth_batch(alg, name, B, rng):
    s = synth_states(name, B, rng)
    a = rng.uniform(-0.99, 0.99, size=(B, alg.action_dim)).astype(np.float32)
    s2 = (s + rng.normal(0, 0.05, size=s.shape)).astype(np.float32)
    r = rng.normal(0, 1, B).astype(np.float32)
    env = alg.real_env
    h = np.asarray(env.get_constraint_values(s2), dtype=np.float32)
    dn = np.asarray(env.check_done(s2)).astype(bool)
    dn[:3] = True
    v = np.asarray(env.check_violation(s2)).astype(bool)
    return [torch.from_numpy(np.ascontiguousarray(x)) for x in (s, a, s2, r, dn, v, h)]


def solver_lrs(sol):
    out = {'critic': sol.critic_optimizer.param_groups[0]['lr'],
           'actor': sol.actor_optimizer.param_groups[0]['lr'],
           'actor_safe': sol.actor_safe_optimizer.param_groups[0]['lr'],
           'multiplier': sol.multiplier_optimizer.param_groups[0]['lr']}
    return np.array([out['critic'], out['actor'], out['actor_safe'], out['multiplier']], dtype=np.float64)


def _changed(sd, prefixes):
    """the snapshot entries of the groups an update step writes (fixture size)"""
    return {k: v for k, v in sd.items() if prefixes is None or k[4:].startswith(prefixes)}


def gen_ssac(out, name, seed, tag, distributional, uncertainty, sac_extra=None, cfg=None, snapshots=None):
    """snapshots: per update, the state-dict prefixes stored after it (None: all keys);
    the full-width fixture keeps the groups each update writes."""
    cfg = cfg or small_config(name, distributional=distributional, uncertainty=uncertainty)
    snap = snapshots or (None, None, None, None)
    if sac_extra:
        cfg.update({'sac_cfg': dict(sac_extra)})
    alg = build_alg(name, cfg, seed)
    sol = alg.solver
    d = meta(name, cfg, alg)
    for k, v in (sac_extra or {}).items():
        d['flag/' + k] = np.array(v)
    rng = np.random.RandomState(seed + 5)
    if uncertainty and not distributional:
        # robust certificate target samples the dynamics model inside update_critic
        # (src/ssac.py:387-400): give it fitted normalizer stats and elites first
        m = alg.model_ensemble
        m.state_normalizer.fit(torch.from_numpy(synth_states(name, 500, rng)))
        m._elite_inds = [2, 0, 1]
        d['model/elite_inds'] = np.array(m._elite_inds)
    d.update(_changed(sd_dict(sol, 'sd0/'), snap[0]))
    d['sd0/log_alpha'] = t2n(sol.log_alpha)
    batch = synth_batch(alg, name, cfg.sac_cfg.batch_size, rng)
    # the reference preprocesses in SMBPO.update_solver; feed preprocessed values directly
    for i, nm in enumerate(['s', 'a', 's2', 'r', 'd', 'v', 'h']):
        d['in/' + nm] = batch[i].numpy()
    with Tape() as tp:
        lq, lqc = sol.update_critic(*batch)
    d.update(tp.to_npz_dict('critic_tape'))
    d['out/lq'], d['out/lqc'] = t2n(lq), t2n(lqc)
    d.update(_changed(sd_dict(sol, 'sd1/'), snap[1]))
    d['lr1'] = solver_lrs(sol)
    with Tape() as tp:
        sol.update_actor_and_alpha(batch[0])
    d.update(tp.to_npz_dict('actor_tape'))
    d.update(_changed(sd_dict(sol, 'sd2/'), snap[2]))
    d['sd2/log_alpha'] = t2n(sol.log_alpha)
    d['lr2'] = solver_lrs(sol)
    with Tape() as tp:
        sol.update_multiplier(batch[0])
    d.update(tp.to_npz_dict('mult_tape'))
    d.update(_changed(sd_dict(sol, 'sd3/'), snap[3]))
    d['lr3'] = solver_lrs(sol)
    np.savez_compressed(os.path.join(out, f'ssac_{tag}.npz'), **d)


# the SSAC configuration branches beside the DRPO default (src/ssac.py:117-161):
# scalar softplus multiplier, fixed temperature, log-alpha temperature loss
SOLVER_FLAG_CASES = [
    ('point-robot', 36, 'scalar_mult_point', True, True, {'mlp_multiplier': False, 'penalty_ub': 1.7}),
    ('quadrotor', 37, 'scalar_mult_quad', False, False, {'mlp_multiplier': False, 'penalty_lb': 0.1}),
    ('quadrotor', 38, 'fixed_alpha_quad', True, True, {'autotune_alpha': False}),
    ('point-robot', 39, 'log_alpha_point', True, True, {'use_log_alpha_loss': True}),
]


def gen_solver_flags(out):
    for name, seed, tag, dist, unc, extra in SOLVER_FLAG_CASES:
        gen_ssac(out, name, seed, tag, dist, unc, extra)


# constrained_fcn='cost' (src/ssac.py:191-195,306-310): the reference runs it with
# distributional_qc=False only, and behind the MLP multiplier only for con_dim == 1
COST_CASES = [
    ('point-robot', 44, 'cost_point', False, True, {'constrained_fcn': 'cost'}),
    ('quadrotor', 45, 'cost_quad', False, False, {'constrained_fcn': 'cost', 'mlp_multiplier': False}),
]


def gen_cost(out):
    for name, seed, tag, dist, unc, extra in COST_CASES:
        gen_ssac(out, name, seed, tag, dist, unc, extra)
    # two rollout_and_update() calls through the device batch path (violation flags
    # gathered from the buffers)
    gen_smbpo_update(out, 'point-robot', 46, 'cost_point', False, {'constrained_fcn': 'cost'})


def gen_fullwidth(out):
    """the reference's DEFAULT widths (actor / critics / certificate /
    multiplier 256, model 200; SMBPO.Config / SSAC.Config defaults), so the 256- and
    200-wide tiling paths meet a reference-held vector directly. SSAC: one update_critic
    + update_actor_and_alpha + update_multiplier at B = 64 (DRPO flags); rollout: B = 64,
    H = 2 at E = 7 / 5 elites. Only the groups each step writes are stored after it."""
    sac_groups = ('actor.', 'actor_safe.', 'critic.', 'critic_target.', 'constraint_critic.',
                  'constraint_critic_target.', 'multiplier.')
    cfg = small_config('quadrotor', E=2, elites=2, model_hidden=200, hidden=256, sac_batch=64)
    gen_ssac(out, 'quadrotor', 81, 'fullwidth_quad', True, True, cfg=cfg,
             snapshots=(sac_groups, ('critic.', 'critic_target.', 'constraint_critic.', 'constraint_critic_target.'),
                        ('actor.', 'actor_safe.'), ('multiplier.',)))
    cfg = small_config('quadrotor', B=64, H=2, E=7, elites=5, model_hidden=200, hidden=256)
    gen_rollout(out, 'quadrotor', 82, cfg=cfg, tag='fullwidth_quad', keep=('solver.actor.', 'model_ensemble.'))


def gen_smbpo_update(out, name, seed, tag=None, distributional=True, sac_extra=None):
    cfg = small_config(name, B=32, H=3, sac_batch=32, distributional=distributional)
    if sac_extra:
        cfg.update({'sac_cfg': dict(sac_extra)})
    alg = build_alg(name, cfg, seed)
    d = meta(name, cfg, alg)
    for k, v in (sac_extra or {}).items():
        d['flag/' + k] = np.array(v)
    d.update(sd_dict(alg, 'sd0/'))
    d['sd0/log_alpha'] = t2n(alg.solver.log_alpha)
    d.update(fill_replay(alg, name, 300, seed + 1, alg.con_dim))
    with Tape() as tp:
        alg.update_models(3)
    d.update(tp.to_npz_dict('fit_tape'))
    d['fit/elite_inds'] = np.array(alg.model_ensemble._elite_inds)
    d.update(sd_dict(alg, 'sd1/'))
    for r in range(2):
        with Tape() as tp:
            alg.rollout_and_update()
        d.update(tp.to_npz_dict(f'rau{r}_tape'))
    d.update(sd_dict(alg, 'sd2/'))
    d['sd2/log_alpha'] = t2n(alg.solver.log_alpha)
    d['lr2'] = solver_lrs(alg.solver)
    d['virt/n'] = np.array(len(alg.virt_buffer))
    for k, v in alg.virt_buffer.get(as_dict=True).items():
        d['virt/' + k] = t2n(v)
    d['losses/critic'] = np.array([float(x) for x in alg.recent_critic_losses])
    d['losses/cons'] = np.array([float(x) for x in alg.recent_cons_critic_losses])
    np.savez_compressed(os.path.join(out, f'smbpo_update_{tag or name}.npz'), **d)


class RecordingPointRobot(PointRobot):
    """The reference PointRobot whose training-env resets (global np.random.uniform,
    src/env/point_robot.py:44-47) are recorded so the test-side env can replay them."""
    resets = []

    def reset(self):
        obs = super().reset()
        if self.id is None:
            RecordingPointRobot.resets.append(np.array(self.state, dtype=np.float64))
        return obs


# run-ablation-1_quadrotor.sh variants (the flags main.py receives via -s):
#   drpo         safe_shield, distributional certificate, linear evaluation shield (run.sh)
#   vanilla      no step shield, vanilla certificate, eval_shield_type 'no' (DRPO-Vanilla, :7-17)
#   shield_only  step shield at threshold 0.0 with the vanilla certificate, linear
#                evaluation shield (DRPO-Shield-only, :31-41)
#   uncert_safe  distributional certificate without the step shield (DRPO-Uncertainty-only,
#                :19-29) evaluated with the 'safe' shield (src/sampling.py:425-428)
TRAINER_VARIANTS = {
    'drpo': dict(safe_shield=True, distributional=True, uncertainty=True, eval_shield_type='linear'),
    'vanilla': dict(safe_shield=False, distributional=False, uncertainty=False, eval_shield_type='no'),
    'shield_only': dict(safe_shield=True, distributional=False, uncertainty=False, eval_shield_type='linear'),
    'uncert_safe': dict(safe_shield=False, distributional=True, uncertainty=True, eval_shield_type='safe'),
}


def trainer_config(seed_cfg, variant='drpo'):
    v = TRAINER_VARIANTS[variant]
    cfg = small_config('point-robot', B=32, H=3, sac_batch=32, distributional=v['distributional'],
                       uncertainty=v['uncertainty'])
    cfg.update({'buffer_min': 40, 'steps_per_epoch': 10, 'model_update_period': 4, 'model_initial_steps': 5,
                'model_steps': 3, 'safe_shield': v['safe_shield'], 'safe_shield_threshold': seed_cfg['shield'],
                'eval_shield_threshold': seed_cfg['eval_shield'], 'eval_shield_type': v['eval_shield_type'],
                'mode': 'train'})
    return cfg


def gen_trainer(out, seed, shield=-0.1, eval_shield=-0.05, variant='drpo'):
    """main.py's loop shape (main.py:50-62): setup() -> evaluate() -> epoch() ->
    evaluate() on point-robot, with every random draw recorded. Shield decisions are
    discrete, so the generator also records how close each shield query came to its
    threshold (the parity test needs a margin well above fp32 noise)."""
    import src.ssac as ssac_mod
    from src.log import default_log as rlog
    cfg = trainer_config({'shield': shield, 'eval_shield': eval_shield}, variant)
    rlog.setup(tempfile.mkdtemp())     # a fresh run dir: episodes.csv holds this run's rows only
    RecordingPointRobot.resets = []
    set_seed(seed)
    factory = lambda id=None: TorchWrapper(RecordingPointRobot(id=id))  # noqa: E731
    data = CheckpointableData()
    alg = SMBPO(cfg, factory, data, 1)
    d = meta('point-robot', cfg, alg)
    d.update(sd_dict(alg, 'sd0/'))
    d['sd0/log_alpha'] = t2n(alg.solver.log_alpha)
    d['cfg/buffer_min'], d['cfg/steps_per_epoch'] = np.array(cfg.buffer_min), np.array(cfg.steps_per_epoch)
    d['cfg/model_update_period'] = np.array(cfg.model_update_period)
    d['cfg/model_initial_steps'], d['cfg/model_steps'] = np.array(cfg.model_initial_steps), np.array(cfg.model_steps)
    d['cfg/shield'], d['cfg/eval_shield'] = np.array(shield), np.array(eval_shield)
    d['cfg/variant'] = np.array(variant)
    for k, v in TRAINER_VARIANTS[variant].items():
        d[f'cfg/{k}'] = np.array(v)
    margins = {'step': [], 'eval': []}
    orig_get_qc = ssac_mod.SSAC._get_qc
    in_eval = [False]
    eval_qc = []          # per evaluation step: the performance-action query, then 11 mixes (linear)

    def rec_get_qc(self, q):
        out_q = orig_get_qc(self, q)
        n = out_q.reshape(-1).shape[0]
        if n == 1 and not in_eval[0]:
            margins['step'].append(float((out_q - shield).abs().min()))
        elif in_eval[0]:
            eval_qc.append(float((out_q - eval_shield).abs().min()))
        return out_q

    def evaluate():
        in_eval[0] = True
        eval_qc.clear()
        try:
            ev = alg.evaluate()
        finally:
            in_eval[0] = False
        # only the queries the shield type decides on (src/sampling.py:422-439)
        etype = cfg.eval_shield_type
        per = 12 if etype == 'linear' else 1
        used = [m for i, m in enumerate(eval_qc) if (etype == 'linear' and i % per != 0) or etype == 'safe']
        margins['eval'].extend(used)
        return ev
    ssac_mod.SSAC._get_qc = rec_get_qc
    try:
        with Tape() as tp:
            alg.setup()
        d.update(tp.to_npz_dict('setup_tape'))
        ev0 = evaluate()
        with Tape() as tp:
            alg.epoch()
        d.update(tp.to_npz_dict('epoch_tape'))
        ev1 = evaluate()
    finally:
        ssac_mod.SSAC._get_qc = orig_get_qc
    keys = sorted(ev0)
    d['eval/keys'] = np.array(keys)
    d['eval/0'] = np.array([ev0[k] for k in keys])
    d['eval/1'] = np.array([ev1[k] for k in keys])
    d['resets'] = np.stack(RecordingPointRobot.resets)
    d['margin/step'] = np.array(margins['step'] or [np.inf])
    d['margin/eval'] = np.array(margins['eval'] or [np.inf])
    d.update(sd_dict(alg, 'sd1/'))
    d['sd1/log_alpha'] = t2n(alg.solver.log_alpha)
    for name, buf in (('replay', alg.replay_buffer), ('virt', alg.virt_buffer)):
        d[f'{name}/n'] = np.array(len(buf))
        for k, v in buf.get(as_dict=True).items():
            d[f'{name}/{k}'] = t2n(v)
    dk = sorted(data._data)
    d['data/keys'] = np.array(dk)
    for i, k in enumerate(dk):
        d[f'data/{i:03d}'] = np.array([np.nan if v is None else float(v) for v in data[k]], dtype=np.float64)
    d['episodes_csv'] = np.array(open(os.path.join(str(rlog.dir), 'episodes.csv')).read())
    print('trainer fixture %s seed %d: min shield margins step %.3g eval %.3g, %d real steps, eval %s / %s' % (
        variant, seed, d['margin/step'].min(), d['margin/eval'].min(), len(alg.replay_buffer), ev0, ev1))
    name = 'trainer_point-robot.npz' if variant == 'drpo' else f'trainer_point-robot_{variant}.npz'
    np.savez_compressed(os.path.join(out, name), **d)
    return float(min(d['margin/step'].min(), d['margin/eval'].min()))


# (step shield threshold, evaluation shield threshold) per variant: Shield-only runs
# the step shield at 0.0 (run-ablation-1_quadrotor.sh:39)
TRAINER_SHIELDS = {'shield_only': (0.0, -0.05)}
# seeds whose shield decisions all clear their thresholds by a margin far above fp32
# noise (printed by gen_trainer; chosen with `make_golden.py trainer <seed> <variant>`)
TRAINER_VARIANT_SEEDS = {'vanilla': 62, 'shield_only': 63, 'uncert_safe': 64}


def gen_fit_epochs(out, name, seed, torch_seed):
    """fit(epochs=1) -> src/train.py::epochal_training (src/dynamics.py:185-194): E
    epochs of torch.randperm minibatches of E*batch_size rows (the last one ragged),
    one Adam step each. The CPU generator is re-seeded with ``torch_seed`` right before
    the call; the build's fit_epochs draws its permutations from the same generator."""
    cfg = small_config(name)
    alg = build_alg(name, cfg, seed)
    model = alg.model_ensemble
    d = meta(name, cfg, alg)
    d.update(sd_dict(model, 'sd/'))
    d.update(fill_replay(alg, name, 1200, seed + 1, alg.con_dim))
    torch.manual_seed(torch_seed)
    d['torch_seed'] = np.array(torch_seed)
    losses = model.fit(alg.replay_buffer, epochs=1)
    d['out/losses'] = np.array(losses, dtype=np.float64)
    d['model/norm_mean'] = t2n(model.state_normalizer.mean)
    d['model/norm_std'] = t2n(model.state_normalizer.std)
    d.update(sd_dict(model, 'fit_sd/'))
    np.savez_compressed(os.path.join(out, f'fit_epochs_{name}.npz'), **d)


def gen_checkpoint(out, seed):
    """A ckpt_{epoch}.pt / data.pt pair written by the reference's own Checkpointer
    (src/checkpoint.py:55-83, main.py:34-35,67-71) from a point-robot SMBPO after a
    short fit + rollout_and_update, stored as raw bytes for the interop test."""
    import io
    from src.checkpoint import Checkpointer
    cfg = small_config('point-robot', B=32, H=3, sac_batch=32)
    alg = build_alg('point-robot', cfg, seed)
    fill_replay(alg, 'point-robot', 300, seed + 1, alg.con_dim)
    alg.update_models(3)
    alg.rollout_and_update()
    alg.epochs_completed += 3
    data = alg.data
    data.append('critic loss', float(alg.recent_critic_losses[-1]))
    data.append('eval return mean', 1.25)
    tmp = tempfile.mkdtemp()
    Checkpointer(alg, tmp, 'ckpt_{}.pt').save(3)
    Checkpointer(data, tmp, 'data.pt').save()
    d = meta('point-robot', cfg, alg)
    d['ckpt_bytes'] = np.frombuffer(open(os.path.join(tmp, 'ckpt_3.pt'), 'rb').read(), dtype=np.uint8)
    d['data_bytes'] = np.frombuffer(open(os.path.join(tmp, 'data.pt'), 'rb').read(), dtype=np.uint8)
    d.update(sd_dict(alg, 'sd/'))
    d['log_alpha'] = t2n(alg.solver.log_alpha)
    np.savez_compressed(os.path.join(out, 'checkpoint_point-robot.npz'), **d)


def gen_init_hashes(out):
    """sha256 of every state_dict tensor of a DEFAULT-width SMBPO (quadrotor dims, E=7)
    for seed 0: pins the build's reference-order initialisation bit-exactly."""
    cfg = copy.deepcopy(SMBPO.Config())
    cfg.update({'sac_cfg': {'qc_under_uncertainty': True, 'distributional_qc': True}})
    alg = build_alg('quadrotor', cfg, 0, epochs=100)
    d = {}
    for k, v in alg.state_dict().items():
        arr = np.ascontiguousarray(t2n(v))
        d['hash/' + k] = np.array(hashlib.sha256(arr.tobytes()).hexdigest())
        d['shape/' + k] = np.array(arr.shape)
        d['dtype/' + k] = np.array(str(arr.dtype))
    d['elite_inds'] = np.array(alg.model_ensemble.elite_inds)
    np.savez_compressed(os.path.join(out, 'init_hashes_quadrotor.npz'), **d)


def main():
    out = HERE
    tmp = tempfile.mkdtemp()
    default_log.setup(tmp)
    if sys.argv[1:2] == ['trainer']:
        seed = int(sys.argv[2]) if len(sys.argv) > 2 else 55
        variant = sys.argv[3] if len(sys.argv) > 3 else 'drpo'
        thr = TRAINER_SHIELDS.get(variant, (-0.1, -0.05))
        gen_trainer(out, seed, thr[0], thr[1], variant)
        return
    if sys.argv[1:2] == ['variants']:
        for variant, seed in TRAINER_VARIANT_SEEDS.items():
            thr = TRAINER_SHIELDS.get(variant, (-0.1, -0.05))
            gen_trainer(out, seed, thr[0], thr[1], variant)
        return
    if sys.argv[1:] == ['fit_epochs']:
        gen_fit_epochs(out, 'quadrotor', 71, 17)
        gen_fit_epochs(out, 'tracking', 72, 18)
        return
    if sys.argv[1:] == ['checkpoint']:
        gen_checkpoint(out, 61)
        return
    if sys.argv[1:] == ['solver_flags']:
        gen_solver_flags(out)
        return
    if sys.argv[1:] == ['cost']:
        gen_cost(out)
        return
    if sys.argv[1:] == ['fullwidth']:
        gen_fullwidth(out)
        return
    if sys.argv[1:] == ['robust']:
        gen_ssac(out, 'quadrotor', 34, 'robust_quad', False, True)
        gen_ssac(out, 'point-robot', 35, 'robust_point', False, True)
        return
    gen_constraints(out)
    gen_init_hashes(out)
    for name, seed in [('point-robot', 11), ('quadrotor', 12)]:
        gen_rollout(out, name, seed)
    for name, seed in [('quadrotor', 21), ('tracking', 22), ('cartpole', 23)]:
        gen_ensemble(out, name, seed)
    gen_ssac(out, 'point-robot', 31, 'drpo_point', True, True)
    gen_ssac(out, 'quadrotor', 32, 'drpo_quad', True, True)
    gen_ssac(out, 'quadrotor', 33, 'vanilla_quad', False, False)
    gen_ssac(out, 'quadrotor', 34, 'robust_quad', False, True)
    gen_ssac(out, 'point-robot', 35, 'robust_point', False, True)
    gen_solver_flags(out)
    gen_cost(out)
    gen_smbpo_update(out, 'point-robot', 41)
    gen_smbpo_update(out, 'quadrotor', 42)
    gen_trainer(out, 55)
    for variant, seed in TRAINER_VARIANT_SEEDS.items():
        thr = TRAINER_SHIELDS.get(variant, (-0.1, -0.05))
        gen_trainer(out, seed, thr[0], thr[1], variant)
    gen_fit_epochs(out, 'quadrotor', 71, 17)
    gen_fit_epochs(out, 'tracking', 72, 18)
    gen_checkpoint(out, 61)
    gen_fullwidth(out)
    print('golden fixtures written to', out)


if __name__ == '__main__':
    main()
