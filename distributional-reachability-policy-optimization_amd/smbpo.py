"""Model-based safe RL trainer (src/smbpo.py:21-440) on the HIP hot path.

The hot path -- rollout (fused per-step kernel, csrc/rollout.hip), update_solver
(SAC engine, sac_step.py) and update_models (ensemble fit) -- runs on the device
with no host synchronisation inside a rollout. Constructor signature, Config
fields, buffers and state_dict layout follow the reference so main.py-style
drivers work unchanged.
"""
import numpy as np
import torch

from .buffers import ConstraintSafetySampleBuffer, DummyModuleWrapper
from .config import BaseConfig, Configurable
from .dynamics import BatchedGaussianEnsemble
from .envs import device_env_params
from .rng import DeviceNoise
from .ssac import SSAC
from .torch_util import Module, device as default_device, pythonic_mean


def env_dims(env):
    import math
    return (int(math.prod(env.observation_space.shape)), int(math.prod(env.action_space.shape)), env.con_dim)


def get_max_episode_steps(env):
    if hasattr(env, '_max_episode_steps'):
        return env._max_episode_steps
    if hasattr(env, 'env'):
        return get_max_episode_steps(env.env)
    raise ValueError('env does not have _max_episode_steps')


class SMBPO(Configurable, Module):
    class Config(BaseConfig):
        sac_cfg = SSAC.Config()
        model_cfg = BatchedGaussianEnsemble.Config()
        model_initial_steps = 10000
        model_steps = 2000
        model_update_period = 250
        save_trajectories = False
        horizon = 10
        alive_bonus = 1.0
        buffer_min = 5000
        buffer_max = 10 ** 6
        steps_per_epoch = 1000
        rollout_batch_size = 100
        solver_updates_per_step = 10
        real_fraction = 0.1
        action_clip_gap = 1e-6
        reward_scale = 1.
        mode = 'train'
        constraint_scale = 10.
        constraint_offset = 0.
        safe_shield = True
        safe_shield_threshold = -0.1
        eval_shield_threshold = -0.05
        eval_shield_type = "linear"

    def __init__(self, config, env_factory, data=None, epochs=1, device=default_device, noise_seed=0):
        Configurable.__init__(self, config)
        Module.__init__(self)
        self.data = data
        self.device = device
        self.env_factory = env_factory
        self.real_env = env_factory()
        self.state_dim, self.action_dim, self.con_dim = env_dims(self.real_env)
        self.env_params = device_env_params(self.real_env)
        assert self.env_params['con_dim'] == self.con_dim, 'env con_dim does not match the device constraint fns'
        self.model_ensemble = BatchedGaussianEnsemble(self.model_cfg, self.state_dim, self.action_dim, device=device)
        self.solver = SSAC(self.sac_cfg, self.state_dim, self.action_dim, self.con_dim, self.horizon, epochs,
                           self.steps_per_epoch, self.solver_updates_per_step, self.constraint_scale, env_factory,
                           self.model_ensemble, device=device)
        self.replay_buffer = self._create_buffer(self.buffer_max)
        self.virt_buffer = self._create_buffer(self.buffer_max)
        self.register_buffer('episodes_sampled', torch.tensor(0, device=device))
        self.register_buffer('steps_sampled', torch.tensor(0, device=device))
        self.register_buffer('n_violations', torch.tensor(0, device=device))
        self.register_buffer('epochs_completed', torch.tensor(0, device=device))
        self.recent_critic_losses = []
        self.recent_cons_critic_losses = []
        self.noise = DeviceNoise(noise_seed)
        self._ws = {}

    @property
    def actor(self):
        return self.solver.actor

    @property
    def constraint_critic(self):
        return self.solver.constraint_critic

    @property
    def actor_safe(self):
        return self.solver.actor_safe

    def _create_buffer(self, capacity):
        buf = ConstraintSafetySampleBuffer(self.state_dim, self.action_dim, capacity, con_dim=self.con_dim,
                                           device=self.device)
        return DummyModuleWrapper(buf)

    def _workspace(self, key, nbytes):
        t = self._ws.get(key)
        if t is None or t.numel() < nbytes:
            t = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=self.device)
            self._ws[key] = t
        return t

    # ------------------------------------------------------------------
    def rollout(self, policy, initial_states=None, noise=None, timer=None):
        """src/smbpo.py:229-249 as one fused kernel per horizon step."""
        from . import ops
        return ops.rollout(self, policy, initial_states, self.noise if noise is None else noise, timer)

    def update_models(self, model_steps, noise=None):
        losses = self.model_ensemble.fit(self.replay_buffer, steps=model_steps,
                                         noise=self.noise if noise is None else noise)
        rewards = self.replay_buffer.get('rewards')
        self.solver.update_r_bounds(rewards.min().item() + self.alive_bonus, rewards.max().item() + self.alive_bonus)
        return losses

    def update_solver(self, update_actor=True, update_multiplier=False, noise=None):
        """src/smbpo.py:251-279: mixed real/virtual minibatch + critic/actor/multiplier updates."""
        eng = self.solver.engine
        noise = self.noise if noise is None else noise
        lq, lqc = eng.update_solver(self, update_actor, update_multiplier, noise)
        self.recent_critic_losses.append(lq)
        self.recent_cons_critic_losses.append(lqc)

    def rollout_and_update(self, noise=None):
        self.rollout(self.actor, noise=noise)
        for step in range(self.solver_updates_per_step):
            self.update_solver(update_actor=step % self.sac_cfg.actor_update_interval == 0,
                               update_multiplier=step % self.sac_cfg.multiplier_update_interval == 0,
                               noise=noise)

    def mean_recent_losses(self):
        return pythonic_mean(self.recent_critic_losses), pythonic_mean(self.recent_cons_critic_losses)
