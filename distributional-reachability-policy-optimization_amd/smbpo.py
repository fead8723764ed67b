"""Model-based safe RL trainer (src/smbpo.py:21-440) on the HIP hot path.

The hot path -- rollout (fused horizon kernel, csrc/rollout.hip), update_solver
(SAC engine, sac_step.py) and update_models (ensemble fit) -- runs on the device
with no host synchronisation inside a rollout. Around it, the trainer keeps the
reference's driver surface so main.py's loop (setup -> evaluate -> epoch ->
evaluate, main.py:29-72) runs against it unchanged:

  step_generator   real-env collection (src/smbpo.py:111-212). The safety shield's
                   decision (qc > threshold -> safe action, :127-136) is taken on the
                   device (drpo_shield_select); the env-info consistency asserts
                   (:158-163) use the device constraint functions.
  setup / epoch    src/smbpo.py:293-325
  evaluate         linear-shield batched evaluation (src/smbpo.py:421-440 ->
                   sampling.sample_episodes_batched): the 11 shield candidates are
                   scored by ONE constraint-critic launch per step.
  log_statistics   src/smbpo.py:327-419 on the stand-alone HIP network forwards.

Constructor signature, Config fields, buffers and state_dict layout follow the
reference; ``noise`` (DeviceNoise by default, TapeNoise for parity replays)
supplies every random draw.
"""
import numpy as np
import torch

from .buffers import ConstraintSafetySampleBuffer, DummyModuleWrapper
from .checkpoint import CheckpointableData
from .config import BaseConfig, Configurable
from .distributed import GradReducer
from .dynamics import BatchedGaussianEnsemble
from .envs import ProductEnv, device_env_params, env_dims, get_max_episode_steps  # noqa: F401
from .log import default_log as log, TabularLog
from .policy import UniformPolicy
from .rng import DeviceNoise
from .ssac import SSAC
from .torch_util import Module, device as default_device, pythonic_mean

N_EVAL_TRAJ = 10
LOSS_AVERAGE_WINDOW = 10
BATCH_MAP_ROWS = 1000      # src/util.py:74 batch_map default


def deciles(a):
    """src/torch_util.py:63-65 (numpy quantiles on the host)."""
    a = a.detach().cpu().numpy() if torch.is_tensor(a) else np.asarray(a)
    q = np.quantile(a, [0.0, 0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 0.9, 1.0])
    return torch.from_numpy(np.asarray(q))


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

    def __init__(self, config, env_factory, data=None, epochs=1, device=default_device, noise_seed=None):
        Configurable.__init__(self, config)
        Module.__init__(self)
        self.data = data if data is not None else CheckpointableData()
        self.device = device
        self.env_factory = env_factory
        self.episode_log = TabularLog(log.dir, 'episodes.csv') if log.dir is not None else None
        self.real_env = env_factory()
        self._eval_env = None
        self.state_dim, self.action_dim, self.con_dim = env_dims(self.real_env)
        # device constraint fns for known envs; None keeps the env's numpy fns (host round trip)
        self.env_params = device_env_params(self.real_env)
        if self.env_params is not None:
            assert self.env_params['con_dim'] == self.con_dim, 'env con_dim does not match the device constraint fns'
        self.model_ensemble = BatchedGaussianEnsemble(self.model_cfg, self.state_dim, self.action_dim, device=device)
        self.solver = SSAC(self.sac_cfg, self.state_dim, self.action_dim, self.con_dim, self.horizon, epochs,
                           self.steps_per_epoch, self.solver_updates_per_step, self.constraint_scale, env_factory,
                           self.model_ensemble, device=device)
        self.replay_buffer = self._create_buffer(self.buffer_max)
        self.virt_buffer = self._create_buffer(self.buffer_max)
        self.uniform_policy = UniformPolicy(self.real_env, device=device)
        self.register_buffer('episodes_sampled', torch.tensor(0, device=device))
        self.register_buffer('steps_sampled', torch.tensor(0, device=device))
        self.register_buffer('n_violations', torch.tensor(0, device=device))
        self.register_buffer('epochs_completed', torch.tensor(0, device=device))
        self.recent_critic_losses = []
        self.recent_cons_critic_losses = []
        self.noise = DeviceNoise(noise_seed)
        self._ws = {}
        self.stepper = None

    @property
    def eval_env(self):
        """ProductEnv of N_EVAL_TRAJ envs (1 in 'test' mode), built on first use
        (the reference builds it in __init__, src/smbpo.py:54-59)."""
        if self._eval_env is None:
            if self.mode == 'train':
                self._eval_env = ProductEnv([self.env_factory(id=i) for i in range(N_EVAL_TRAJ)])
            elif self.mode == 'test':
                self._eval_env = ProductEnv([self.env_factory(id=i) for i in range(1)])
            else:
                raise ValueError(f'Invalid SMBPO mode {self.mode!r}')
        return self._eval_env

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

    def _log_tabular(self, row):
        for k, v in row.items():
            self.data.append(k, v, verbose=True)
        if self.episode_log is not None:
            self.episode_log.row(row)

    # ------------------------------------------------------------------ constraint checks
    def check_constraints(self, states):
        """(done, violation, constraint_value) of a batch of states: the device constraint
        functions for known envs, else the env's numpy functions (src/smbpo.py:63-65)."""
        from . import ops
        if self.env_params is not None:
            return ops.env_constraints(self.env_params, states)
        from .torch_util import torchify
        s = states.detach().cpu().numpy()
        env = self.real_env
        return (torchify(env.check_done(s)), torchify(env.check_violation(s)),
                torchify(env.get_constraint_values(s)))

    def _shielded_action(self, state, noise):
        """actor.act1 + the real-env safety shield (src/smbpo.py:124-136); the shield's
        branch is a per-row select on the device."""
        from . import ops
        action = self.actor.act1(state, eval=False, noise=noise)
        if not self.safe_shield:
            return action
        sol = self.solver
        q = self.constraint_critic(state.unsqueeze(0), action.unsqueeze(0), uncertainty=sol.distributional_qc,
                                   noise=noise)
        a_safe = self.actor_safe.act(state.unsqueeze(0), eval=True)
        return ops.shield_select(q.reshape(1, -1), ops.SHIELD_THRESHOLD, self.safe_shield_threshold,
                                 action.unsqueeze(0), a_safe)[0]

    # ------------------------------------------------------------------ real-env collection
    def step_generator(self):
        """src/smbpo.py:111-212: one real-env step per next(); after buffer_min every
        step runs update_models (every model_update_period steps) and
        rollout_and_update() before acting."""
        max_episode_steps = get_max_episode_steps(self.real_env)
        episode = self._create_buffer(max_episode_steps)
        state = self.real_env.reset()
        while True:
            noise = self.noise.collection()   # identical on every data-parallel rank
            t = int(self.steps_sampled.item())
            if t >= self.buffer_min:
                if t % self.model_update_period == 0:
                    self.update_models(self.model_steps)
                self.rollout_and_update()
                action = self._shielded_action(state, noise)
            else:
                action = self.uniform_policy.act1(state, eval=False, noise=noise)
            next_state, reward, done, info = self.real_env.step(action)
            violation = info['violation']
            constraint_value = torch.tensor(info['constraint_value'], dtype=torch.float)
            d_chk, v_chk, h_chk = self.check_constraints(torch.as_tensor(next_state).unsqueeze(0))
            d_chk, v_chk, h_chk = bool(d_chk.reshape(-1)[0]), bool(v_chk.reshape(-1)[0]), h_chk.reshape(-1).cpu()
            assert done == d_chk, (done, d_chk, next_state)
            assert violation == v_chk, (violation, v_chk, next_state)
            assert torch.all(torch.isclose(constraint_value.reshape(-1), h_chk, atol=1e-03)), \
                (constraint_value, h_chk)
            for buffer in (episode, self.replay_buffer):
                buffer.append(states=state, actions=action, next_states=next_state, rewards=reward, dones=done,
                              violations=violation, constraint_values=constraint_value)
            self.steps_sampled += 1

            if done or len(episode) == max_episode_steps:
                episode_return = episode.get('rewards').sum().item()
                episode_length = len(episode)
                episode_safe = not episode.get('violations').any()
                self.episodes_sampled += 1
                if not episode_safe:
                    self.n_violations += episode.get('violations').sum()
                self._log_tabular({
                    'episodes sampled': self.episodes_sampled.item(),
                    'total violations': self.n_violations.item(),
                    'steps sampled': self.steps_sampled.item(),
                    'collect return': episode_return,
                    'collect return (+bonus)': episode_return + episode_length * self.alive_bonus,
                    'collect length': episode_length,
                    'collect safe': episode_safe,
                })
                if self.save_trajectories:
                    raise NotImplementedError('save_trajectories (h5py episode files) is outside the hot path; '
                                              'the reference writes them with src/sampling.py:202')
                episode = self._create_buffer(max_episode_steps)
                state = self.real_env.reset()
            else:
                if self.steps_sampled % max_episode_steps == 0:
                    self._log_tabular({
                        'episodes sampled': self.episodes_sampled.item(),
                        'total violations': self.n_violations.item(),
                        'steps sampled': self.steps_sampled.item(),
                        'collect return': None,
                        'collect return (+bonus)': None,
                        'collect length': None,
                        'collect safe': None,
                    })
                state = next_state
            yield t

    # ------------------------------------------------------------------ hot path
    def rollout(self, policy, initial_states=None, noise=None, timer=None):
        """src/smbpo.py:229-249 as one fused kernel for the whole horizon (device
        constraint fns), or per-step launches around the env's host fns otherwise."""
        from . import ops
        noise = self.noise if noise is None else noise
        if self.env_params is None:
            return ops.rollout_host_env(self, policy, initial_states, noise)
        return ops.rollout(self, policy, initial_states, noise, timer)

    def update_models(self, model_steps, noise=None):
        """src/smbpo.py:214-227."""
        log.message(f'Fitting models @ t = {self.steps_sampled.item()}')
        losses = self.model_ensemble.fit(self.replay_buffer, steps=model_steps,
                                         noise=self.noise if noise is None else noise)
        if len(losses):
            log.message('Loss statistics:')
            log.message(f'\tFirst {LOSS_AVERAGE_WINDOW}: {np.mean(losses[:LOSS_AVERAGE_WINDOW])}')
            log.message(f'\tLast {LOSS_AVERAGE_WINDOW}: {np.mean(losses[-LOSS_AVERAGE_WINDOW:])}')
            log.message(f'\tDeciles: {deciles(losses)}')
        rewards = self.replay_buffer.get('rewards')
        bounds = torch.stack([rewards.min(), rewards.max()]).float()
        GradReducer().broadcast_(bounds)     # data parallel: rank 0's bounds on every replica
        r_min, r_max = bounds.tolist()
        self.solver.update_r_bounds(r_min + self.alive_bonus, r_max + self.alive_bonus)
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

    # ------------------------------------------------------------------ driver surface
    def setup(self):
        """src/smbpo.py:293-319: collect buffer_min uniform-policy steps, then the
        initial model fit."""
        if self.save_trajectories:
            raise NotImplementedError('save_trajectories (h5py episode files) is outside the hot path')
        if self.episodes_sampled.item() > 0:
            raise NotImplementedError('reloading collected episodes needs the h5py episode files '
                                      '(src/smbpo.py:298-303, save_trajectories), which are outside the hot path')
        assert len(self.replay_buffer) == self.steps_sampled
        self.stepper = self.step_generator()
        if len(self.replay_buffer) < self.buffer_min:
            log.message('Collecting initial data')
            while len(self.replay_buffer) < self.buffer_min:
                next(self.stepper)
            log.message('Initial model training')
            self.update_models(self.model_initial_steps)
        log.message('Collecting initial virtual data')
        log.message('Setup done!')

    def epoch(self):
        """src/smbpo.py:321-325."""
        if self.stepper is None:
            self.stepper = self.step_generator()
        for _ in range(self.steps_per_epoch):
            next(self.stepper)
        self.log_statistics()
        self.epochs_completed += 1

    def evaluate(self):
        """src/smbpo.py:421-440: N_EVAL_TRAJ shielded evaluation episodes."""
        from .sampling import sample_episodes_batched
        trajs = sample_episodes_batched(self.eval_env, self.solver, N_EVAL_TRAJ, eval=True,
                                        safe_shield_threshold=self.eval_shield_threshold,
                                        shield_type=self.eval_shield_type)
        lengths = [len(t) for t in trajs]
        returns = [t.get('rewards').sum().item() for t in trajs]
        violations = [t.get('violations').sum().item() for t in trajs]
        return {
            'eval return mean': float(np.mean(returns)),
            'eval return std': float(np.std(returns)),
            'eval length mean': float(np.mean(lengths)),
            'eval length std': float(np.std(lengths)),
            'eval violation mean': float(np.mean(violations)),
        }

    # ------------------------------------------------------------------ diagnostics
    def evaluate_models(self):
        """src/smbpo.py:327-336: per-member normalised one-step error deciles over the
        real buffer (one all-member forward, member stride 0 for the shared rows)."""
        states, actions, next_states = self.replay_buffer.get('states', 'actions', 'next_states')
        state_std = states.std(dim=0)
        state_std[state_std < 1e-7] = 1.0
        with torch.no_grad():
            predicted = self.model_ensemble.means(states, actions)[0]
        for i in range(self.model_cfg.ensemble_size):
            errors = torch.norm((predicted[i] - next_states) / (state_std + 1e-7), dim=1)
            log.message(f'Model {i + 1} error deciles: {deciles(errors)}')

    def _consume_chunk_draws(self, n, noise):
        """The reference's constraint_critic(sample=True) draws one randn_like per
        batch_map chunk of 1000 rows (src/smbpo.py:376-378, src/ssac.py:80); a recorded
        tape keeps those draws in order (they do not affect the std it reports)."""
        C = self.con_dim
        for s0 in range(0, n, BATCH_MAP_ROWS):
            m = min(BATCH_MAP_ROWS, n - s0)
            noise.randn_like((m, C) if C > 1 else (m,), used=False)

    def log_statistics(self):
        """src/smbpo.py:338-419."""
        from .sampling import stat_forwards
        self.evaluate_models()
        avg = pythonic_mean(self.recent_critic_losses) if self.recent_critic_losses else None
        log.message(f'Average recent critic loss: {avg}')
        self.data.append('critic loss', avg)
        self.recent_critic_losses.clear()
        avg = pythonic_mean(self.recent_cons_critic_losses) if self.recent_cons_critic_losses else None
        log.message(f'Average recent constraint critic loss: {avg}')
        self.data.append('constraint critic loss', avg)
        self.recent_cons_critic_losses.clear()
        log.message('Buffer sizes:')
        log.message(f'\tReal: {len(self.replay_buffer)}')
        log.message(f'\tVirtual: {len(self.virt_buffer)}')

        noise = self.noise
        real_s, real_a, real_v = self.replay_buffer.get('states', 'actions', 'violations')
        virt_s, virt_v = self.virt_buffer.get('states', 'violations')
        virt_a = self.actor.act(virt_s, eval=True).detach()
        groups = {
            'real (violation)': (real_s[real_v], real_a[real_v]),
            'real (~violation)': (real_s[~real_v], real_a[~real_v]),
            'virtual (violation)': (virt_s[virt_v], virt_a[virt_v]),
            'virtual (~violation)': (virt_s[~virt_v], virt_a[~virt_v]),
        }
        cfg = self.sac_cfg
        for which, (states, actions) in groups.items():
            mean_q = mean_qc = mean_qc_std = mean_lam = None
            if len(states) > 0:
                if cfg.distributional_qc and noise.parity:
                    self._consume_chunk_draws(len(states), noise)
                st = stat_forwards(self.solver, states, actions, cfg.distributional_qc, cfg.mlp_multiplier)
                mean_q, mean_qc = st['q'].mean(), st['qc'].mean()
                if cfg.distributional_qc:
                    mean_qc_std = st['qc_std'].mean()
                if 'lam' in st:
                    mean_lam = st['lam'].mean()
            log.message(f'Average Q {which}: {mean_q}')
            self.data.append(f'Average Q {which}', mean_q)
            log.message(f'Average Qc {which}: {mean_qc}')
            self.data.append(f'Average Qc {which}', mean_qc)
            if cfg.distributional_qc:
                log.message(f'Average Qc std {which}: {mean_qc_std}')
                self.data.append(f'Average Qc std {which}', mean_qc_std)
            if cfg.mlp_multiplier:
                log.message(f'Average Lambda {which}: {mean_lam}')
                self.data.append(f'Average Lambda {which}', mean_lam)
        if not cfg.mlp_multiplier:
            mean_lam = self.solver.lam.item()
            log.message(f'Average Lambda: {mean_lam}')
            self.data.append('Average Lambda', mean_lam)
        if torch.cuda.is_available():
            t = torch.cuda.get_device_properties(0).total_memory
            r, a = torch.cuda.memory_reserved(0), torch.cuda.memory_allocated(0)
            log.message(f'GPU memory info: total {t}, reserved {r}, allocated {a}, '
                        f'reserved but unallocated {r - a}')

    def mean_recent_losses(self):
        return pythonic_mean(self.recent_critic_losses), pythonic_mean(self.recent_cons_critic_losses)
