"""Test-side point-robot environment for the trainer parity test.

A restatement of the reference's unicycle point-robot task
(src/env/point_robot.py:7-176: 11-d observation, 2 hazards of radius 0.8, goal
disc of radius 0.3 at (2.2, 2.2), dt 0.05, 300 steps) using the same numpy
operations, so a trajectory driven by the same actions is reproduced to fp32/fp64
rounding. The training env (id None) replays the initial states recorded by
tests/golden/make_golden.py (the reference draws them from the global numpy RNG);
evaluation envs (id set) start from the fixed state, as the reference does.

TorchEnv plays the reference's TorchWrapper (src/env/torch_wrapper.py): tensors
on the device in, device tensors out.
"""
import numpy as np
import torch

from drpo_amd.envs import Box

HAZARDS = (np.array([0.4, -1.2]), np.array([-0.4, 1.2]))
HAZARD_SIZE, GOAL, GOAL_SIZE, DT = 0.8, np.array([2.2, 2.2]), 0.3, 0.05


class PointRobot:
    def __init__(self, id=None, resets=None):
        self.observation_space = Box(-np.inf, np.inf, (11,))
        self.action_space = Box(-1.0, 1.0, (2,))
        self.id = id
        self.resets = resets
        self.state = None
        self.last_dist = None
        self.con_dim = 1
        self._max_episode_steps = 300

    # --- dynamics ---------------------------------------------------------
    @staticmethod
    def _rates(s, u):
        v, th = s[2], s[3]
        return np.array([v * np.cos(th), v * np.sin(th), u[0], u[1]], dtype=np.float32)

    def _observe(self):
        st = self.state
        o = np.zeros(11, dtype=np.float32)
        o[:3] = st[:3]
        c, s = np.cos(st[3]), np.sin(st[3])
        o[3], o[4] = c, s
        rot = np.array([[c, -s], [s, c]], dtype=np.float32)
        for i, hz in enumerate(HAZARDS):
            x, y = (hz[:2] - st[:2]) @ rot
            z = x + 1j * y
            o[5 + 3 * i] = np.abs(z)
            ang = np.angle(z)
            o[6 + 3 * i], o[7 + 3 * i] = np.cos(ang), np.sin(ang)
        return o

    def reset(self):
        if self.id is not None:
            self.state = np.array([-2.5, -2.5, 2.0, np.pi / 4], dtype=np.float32)
        else:
            self.state = np.array(self.resets.pop(0), dtype=np.float64)
        self.last_dist = np.linalg.norm([self.state[0] - GOAL[0], self.state[1] - GOAL[1]])
        return self._observe()

    def step(self, action):
        action = np.clip(action, self.action_space.low, self.action_space.high)
        st = self.state + self._rates(self.state, action) * DT
        dist = np.linalg.norm([st[0] - GOAL[0], st[1] - GOAL[1]])
        reward = 0.0 + (self.last_dist - dist)
        self.last_dist = dist
        done = False
        if dist <= GOAL_SIZE:
            reward += 1
            done = True
        if abs(st[0]) > 3.0 or abs(st[1]) > 3.0:
            done = True
        md = float('inf')
        for hz in HAZARDS:
            md = min(np.linalg.norm(hz[:2] - st[:2]), md)
        h = HAZARD_SIZE - md
        info = dict(cost=int(h <= 0), constraint_value=h, violation=(h > 0).item())
        self.state = st
        return self._observe(), reward, done, info

    # --- batched checks on the host (what the reference env exposes) -------
    def get_constraint_values(self, states):
        states = np.atleast_2d(states)
        md = np.full(states.shape[0], float('inf'))
        for hz in HAZARDS:
            md = np.minimum(np.linalg.norm(hz[:2] - states[:, :2], axis=1), md)
        return HAZARD_SIZE - np.squeeze(md)

    def check_violation(self, states):
        return self.get_constraint_values(np.atleast_2d(states)) > 0

    def check_done(self, states):
        states = np.atleast_2d(states)
        oob = (states[:, 0] < -3.0) | (states[:, 0] > 3.0) | (states[:, 1] < -3.0) | (states[:, 1] > 3.0)
        goal = np.linalg.norm(states[:, :2] - GOAL, axis=1) <= GOAL_SIZE
        done = oob | goal
        return done.item() if done.ndim == 0 else done


class TorchEnv:
    """numpy env <-> device tensors (src/env/torch_wrapper.py:6-11)."""

    def __init__(self, env, device):
        self.env = env
        self.device = device

    def __getattr__(self, name):
        if name.startswith('__'):
            raise AttributeError(name)
        return getattr(self.__dict__['env'], name)

    def reset(self):
        return torch.as_tensor(self.env.reset()).to(self.device)

    def step(self, action):
        a = action.detach().cpu().numpy() if torch.is_tensor(action) else np.asarray(action)
        obs, r, d, info = self.env.step(a)
        return torch.as_tensor(obs).to(self.device), float(r), d, info
