"""Shape-only stand-ins for the reference env classes (the build recognises envs by
class name; the real classes need gym / mujoco / safe_control_gym). Constraint
functions are evaluated on the device, so these carry only dims."""
import numpy as np


class _Space:
    def __init__(self, shape, low=None, high=None):
        self.shape = tuple(shape)
        self.low = low
        self.high = high


class _Env:
    S, A, C, T = 1, 1, 1, 100

    def __init__(self, id=None):
        self.observation_space = _Space((self.S,))
        self.action_space = _Space((self.A,), -np.ones(self.A), np.ones(self.A))
        self.con_dim = self.C
        self._max_episode_steps = self.T


class PointRobot(_Env):
    S, A, C, T = 11, 2, 1, 300


class QuadrotorWrapperEnv(_Env):
    S, A, C, T = 12, 2, 2, 360
    x_threshold, z_threshold = 2.0, 3.0


class SafeInvertedPendulumEnv(_Env):
    S, A, C, T = 4, 1, 4, 1000


class SimuVeh3dofcontiSurrCstr(_Env):
    S, A, C, T = 51, 2, 1, 200
    surr_vehs_start_dim, surr_veh_num = 47, 1


ENVS = {'point-robot': PointRobot, 'quadrotor': QuadrotorWrapperEnv, 'cartpole': SafeInvertedPendulumEnv,
        'tracking': SimuVeh3dofcontiSurrCstr}
