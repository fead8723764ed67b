"""Device environment registry: maps the reference's env classes to the batched
constraint functions implemented on the device (csrc/env_constraints.hpp).

The reference calls env.check_done / check_violation / get_constraint_values on
host numpy arrays (src/smbpo.py:63-65); the build evaluates the same functions
inside the fused rollout kernel. Envs are recognised by class name (the
reference's classes need gym / mujoco / safe_control_gym, which the build does not
import) or by an explicit ``drpo_env_id`` attribute."""
import numpy as np

ENV_IDS = {'PointRobot': 0, 'QuadrotorWrapperEnv': 1, 'SafeInvertedPendulumEnv': 2,
           'SimuVeh3dofcontiSurrCstr': 3}
ENV_NAMES = {'point-robot': 0, 'quadrotor': 1, 'cartpole': 2, 'cartpole-move': 2, 'cartpole-upright': 2,
             'tracking': 3}
CON_DIM = {0: 1, 1: 2, 2: 4, 3: 1}
QUAD_X_THRESHOLD, QUAD_Z_THRESHOLD = 2.0, 3.0   # safe_control_gym defaults (unpinned)
CART_X_THRESHOLD, CART_TH_THRESHOLD = 0.9, 0.2   # SafeInvertedPendulumEnv defaults (inverted_pendulum.py:11-16)


def _unwrap(env):
    seen = 0
    while env is not None and seen < 8:
        if hasattr(env, 'drpo_env_id') or type(env).__name__ in ENV_IDS:
            return env
        env = getattr(env, 'env', None)
        seen += 1
    return None


def device_env_params(env, required=False):
    """dict(env_id, con_dim, tracking_surr_start, tracking_n_surr, thr0, thr1) for an env
    with device constraint functions, or None for an unknown env: the trainer then
    keeps the reference's host numpy round trip (src/smbpo.py:63-65) for it.

    thr0/thr1: quadrotor x/z_threshold (safe_control_gym attributes, unpinned
    defaults 2/3); cartpole x_threshold / th_threshold
    (src/env/poles/inverted_pendulum.py:11-17, kwarg ``threshold``)."""
    if isinstance(env, str):
        eid, e = ENV_NAMES[env], None
    else:
        e = _unwrap(env)
        if e is None:
            if required:
                raise NotImplementedError(f'no device constraint functions for env {type(env).__name__}; '
                                          f'known: {sorted(ENV_IDS)}')
            return None
        eid = getattr(e, 'drpo_env_id', None)
        eid = ENV_IDS[type(e).__name__] if eid is None else int(eid)
    p = dict(env_id=eid, con_dim=CON_DIM[eid], tracking_surr_start=47, tracking_n_surr=1, thr0=0.0, thr1=0.0)
    if eid == 1:
        p['thr0'], p['thr1'] = QUAD_X_THRESHOLD, QUAD_Z_THRESHOLD
    if eid == 2:
        p['thr0'], p['thr1'] = CART_X_THRESHOLD, CART_TH_THRESHOLD
    if e is not None and eid == 3:
        p['tracking_surr_start'] = int(getattr(e, 'surr_vehs_start_dim', 47))
        p['tracking_n_surr'] = int(getattr(e, 'surr_veh_num', 1))
    if e is not None and eid == 1:
        inner = getattr(e, 'env', e)
        p['thr0'] = float(getattr(inner, 'x_threshold', QUAD_X_THRESHOLD))
        p['thr1'] = float(getattr(inner, 'z_threshold', QUAD_Z_THRESHOLD))
    if e is not None and eid == 2:
        p['thr0'] = float(getattr(e, 'x_threshold', CART_X_THRESHOLD))
        p['thr1'] = float(getattr(e, 'th_threshold', CART_TH_THRESHOLD))
    return p


class Box:
    """Minimal continuous space (gym.spaces.Box surface used by the trainer: shape,
    low, high) for dims-only and test environments."""

    def __init__(self, low, high, shape=None, dtype=np.float32):
        if shape is None:
            shape = np.shape(low)
        self.shape = tuple(shape)
        self.dtype = dtype
        self.low = np.broadcast_to(np.asarray(low, dtype), self.shape).copy()
        self.high = np.broadcast_to(np.asarray(high, dtype), self.shape).copy()


_Space = Box


class ShapeEnv:
    """Dims-only stand-in for a reference env class (synthetic benchmarks and tests):
    the device constraint functions are selected by env id, so no simulator is needed."""

    DIMS = {0: (11, 2, 300), 1: (12, 2, 360), 2: (4, 1, 1000), 3: (51, 2, 200)}

    def __init__(self, name, id=None):
        self.drpo_env_id = ENV_NAMES[name]
        S, A, T = self.DIMS[self.drpo_env_id]
        self.observation_space = Box(-np.inf, np.inf, (S,))
        self.action_space = Box(-1.0, 1.0, (A,))
        self.con_dim = CON_DIM[self.drpo_env_id]
        self._max_episode_steps = T
        if self.drpo_env_id == 3:
            self.surr_vehs_start_dim, self.surr_veh_num = 47, 1
        if self.drpo_env_id == 1:
            self.x_threshold, self.z_threshold = QUAD_X_THRESHOLD, QUAD_Z_THRESHOLD
        if self.drpo_env_id == 2:
            self.x_threshold, self.th_threshold = CART_X_THRESHOLD, CART_TH_THRESHOLD


def get_max_episode_steps(env):
    """src/env/util.py:27-33."""
    if hasattr(env, '_max_episode_steps'):
        return env._max_episode_steps
    if hasattr(env, 'env'):
        return get_max_episode_steps(env.env)
    raise ValueError('env does not have _max_episode_steps')


def env_dims(env):
    """src/env/util.py:23-24 (Box spaces: prod(shape))."""
    import math
    return (int(math.prod(env.observation_space.shape)), int(math.prod(env.action_space.shape)), env.con_dim)


class ProductEnv:
    """Batch of independent host environments (src/env/batch.py:87-109) for evaluation.

    States live on the device (the envs' TorchWrapper returns device tensors); the
    actions of one step are copied to the host ONCE and each env steps on its row
    (the reference copies per env)."""

    def __init__(self, envs, max_episode_steps=None):
        self.envs = list(envs)
        self.proto_env = self.envs[0]
        self.n_envs = len(self.envs)
        self._max_episode_steps = max_episode_steps if max_episode_steps is not None else \
            get_max_episode_steps(self.proto_env)

    @property
    def observation_space(self):
        return self.proto_env.observation_space

    @property
    def action_space(self):
        return self.proto_env.action_space

    @property
    def con_dim(self):
        return self.proto_env.con_dim

    def partial_reset(self, indices):
        import torch
        return torch.stack([self.envs[int(i)].reset() for i in indices])

    def reset(self):
        return self.partial_reset(range(self.n_envs))

    def step(self, actions):
        import torch
        acts = actions.detach().cpu() if torch.is_tensor(actions) else actions
        next_states, rewards, dones, infos = [], [], [], []
        for env, a in zip(self.envs, acts):
            s2, r, d, info = env.step(a)
            next_states.append(s2)
            rewards.append(r)
            dones.append(d)
            infos.append(info)
        dev = next_states[0].device
        return (torch.stack(next_states), torch.tensor(rewards, device=dev), torch.tensor(dones, device=dev),
                infos)

    def __repr__(self):
        return f'Batch<{self.n_envs}x{self.proto_env}>'
