"""Device environment registry: maps the reference's env classes to the batched
constraint functions implemented on the device (csrc/env_constraints.hpp).

The reference calls env.check_done / check_violation / get_constraint_values on
host numpy arrays (src/smbpo.py:63-65); the build evaluates the same functions
inside the fused rollout kernel. Envs are recognised by class name (the
reference's classes need gym / mujoco / safe_control_gym, which the build does not
import) or by an explicit ``drpo_env_id`` attribute."""
ENV_IDS = {'PointRobot': 0, 'QuadrotorWrapperEnv': 1, 'SafeInvertedPendulumEnv': 2,
           'SimuVeh3dofcontiSurrCstr': 3}
ENV_NAMES = {'point-robot': 0, 'quadrotor': 1, 'cartpole': 2, 'cartpole-move': 2, 'cartpole-upright': 2,
             'tracking': 3}
CON_DIM = {0: 1, 1: 2, 2: 4, 3: 1}
QUAD_X_THRESHOLD, QUAD_Z_THRESHOLD = 2.0, 3.0   # safe_control_gym defaults (unpinned)


def _unwrap(env):
    seen = 0
    while env is not None and seen < 8:
        if hasattr(env, 'drpo_env_id') or type(env).__name__ in ENV_IDS:
            return env
        env = getattr(env, 'env', None)
        seen += 1
    return None


def device_env_params(env):
    """dict(env_id, con_dim, tracking_surr_start, tracking_n_surr, quad_x/z_threshold)."""
    if isinstance(env, str):
        eid, e = ENV_NAMES[env], None
    else:
        e = _unwrap(env)
        if e is None:
            raise NotImplementedError(f'no device constraint functions for env {type(env).__name__}; '
                                      f'known: {sorted(ENV_IDS)}')
        eid = getattr(e, 'drpo_env_id', None)
        eid = ENV_IDS[type(e).__name__] if eid is None else int(eid)
    p = dict(env_id=eid, con_dim=CON_DIM[eid], tracking_surr_start=47, tracking_n_surr=1,
             quad_x_threshold=QUAD_X_THRESHOLD, quad_z_threshold=QUAD_Z_THRESHOLD)
    if e is not None and eid == 3:
        p['tracking_surr_start'] = int(getattr(e, 'surr_vehs_start_dim', 47))
        p['tracking_n_surr'] = int(getattr(e, 'surr_veh_num', 1))
    if e is not None and eid == 1:
        inner = getattr(e, 'env', e)
        p['quad_x_threshold'] = float(getattr(inner, 'x_threshold', QUAD_X_THRESHOLD))
        p['quad_z_threshold'] = float(getattr(inner, 'z_threshold', QUAD_Z_THRESHOLD))
    return p


class _Space:
    def __init__(self, shape):
        self.shape = tuple(shape)


class ShapeEnv:
    """Dims-only stand-in for a reference env class (synthetic benchmarks and tests):
    the device constraint functions are selected by env id, so no simulator is needed."""

    DIMS = {0: (11, 2, 300), 1: (12, 2, 360), 2: (4, 1, 1000), 3: (51, 2, 200)}

    def __init__(self, name, id=None):
        self.drpo_env_id = ENV_NAMES[name]
        S, A, T = self.DIMS[self.drpo_env_id]
        self.observation_space = _Space((S,))
        self.action_space = _Space((A,))
        self.con_dim = CON_DIM[self.drpo_env_id]
        self._max_episode_steps = T
        if self.drpo_env_id == 3:
            self.surr_vehs_start_dim, self.surr_veh_num = 47, 1
        if self.drpo_env_id == 1:
            self.x_threshold, self.z_threshold = QUAD_X_THRESHOLD, QUAD_Z_THRESHOLD
