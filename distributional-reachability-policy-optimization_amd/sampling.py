"""Shielded batched evaluation and the per-epoch network statistics.

sample_episodes_batched (src/sampling.py:409-464) with the evaluation shields on
the device: per environment step the performance and safe actors run one fused
forward each, the linear shield's 11 candidate actions are built by
drpo_shield_mix and scored by ONE constraint-critic launch over 11*n rows
(the reference makes 11 calls), and drpo_shield_select picks each row's action.
Only the chosen actions cross to the host, once per step, for the envs.

stat_forwards: the Q / Qc / Qc-std / lambda forwards of SMBPO.log_statistics
(src/smbpo.py:355-399) over a whole row set in single launches (the reference
maps them over 1000-row chunks).
"""
import torch

from . import ops
from .buffers import SafetySampleBuffer
from .envs import ProductEnv, env_dims
from .rng import DeviceNoise

LINEAR_SHIELD_CANDIDATES = 11       # ratio (10 - i) / 10, i = 0..10 (src/sampling.py:432-434)
_NO_TAPE = DeviceNoise(0, rank=0)   # draws the reference makes but whose values are unused


class _Trajectory:
    """Rows of one evaluation episode, kept as device row tensors until it completes."""

    def __init__(self):
        self.rows = []

    def __len__(self):
        return len(self.rows)

    def to_buffer(self, S, A, capacity, device):
        buf = SafetySampleBuffer(S, A, capacity, device=device)
        if self.rows:
            cols = list(zip(*self.rows))
            buf.extend(states=torch.stack(cols[0]), actions=torch.stack(cols[1]), next_states=torch.stack(cols[2]),
                       rewards=torch.stack(cols[3]), dones=torch.stack(cols[4]),
                       violations=torch.tensor(cols[5], dtype=torch.bool, device=device))
        return buf


def shielded_actions(policy, states, eval, safe_shield_threshold, shield_type, noise=None):
    """The action selection of one evaluation step (src/sampling.py:422-439)."""
    a_perf = policy.act(states, eval=eval, noise=noise) if noise is not None else policy.act(states, eval=eval)
    if not eval or shield_type not in ('safe', 'linear'):
        return a_perf
    a_safe = policy.actor_safe.act(states, eval=eval)
    cc = policy.constraint_critic
    if shield_type == 'safe':
        q = cc(states, a_perf)
        return ops.shield_select(q.reshape(len(states), -1), ops.SHIELD_THRESHOLD, safe_shield_threshold, a_perf,
                                 a_safe)
    K = LINEAR_SHIELD_CANDIDATES
    mixes = ops.shield_mix(a_perf, a_safe, K)
    q = ops.constraint_critic_forward(cc, states, mixes.reshape(K * len(states), -1), repeat=K)
    return ops.shield_select(q.reshape(K * len(states), -1), ops.SHIELD_LINEAR, safe_shield_threshold, a_perf,
                             a_safe, mixes)


def sample_episodes_batched(env, policy, n_traj, eval=False, safe_shield_threshold=-0.1, shield_type="linear"):
    """src/sampling.py:409-464: step a batch of envs until n_traj episodes complete;
    returns their SafetySampleBuffers in completion order."""
    if not hasattr(env, 'n_envs'):
        env = ProductEnv([env])
    S, A, _ = env_dims(env)
    T = env._max_episode_steps
    trajs = [_Trajectory() for _ in range(env.n_envs)]
    complete = []
    states = env.reset()
    dev = states.device
    while True:
        actions = shielded_actions(policy, states, eval, safe_shield_threshold, shield_type)
        next_states, rewards, dones, infos = env.step(actions)
        violations = [bool(info['violation']) for info in infos]
        _next_states = next_states.clone()
        reset_indices = []
        dones_h = dones.cpu().tolist()
        for i in range(env.n_envs):
            trajs[i].rows.append((states[i], actions[i], next_states[i], rewards[i], dones[i], violations[i]))
            if dones_h[i] or len(trajs[i]) == T:
                complete.append(trajs[i].to_buffer(S, A, T, dev))
                if len(complete) == n_traj:
                    return complete
                reset_indices.append(i)
                trajs[i] = _Trajectory()
        if reset_indices:
            _next_states[reset_indices] = env.partial_reset(reset_indices)
        states = _next_states


def stat_forwards(solver, states, actions, distributional, mlp_multiplier):
    """Q / Qc / Qc-std / lambda of SMBPO.log_statistics (src/smbpo.py:369-399) for one
    row set: critic mean, constraint-critic mean (max over C), its std, the safe actor's
    certificate and the multiplier on it. The cost certificate reports its raw mean and
    no lambda (the reference's reachability-only branches, src/smbpo.py:380-398)."""
    out = {'q': solver.critic.mean(states, actions)}
    cc = solver.constraint_critic
    reach = solver.constrained_fcn == 'reachability'
    qc = cc(states, actions)
    out['qc'] = solver._get_qc(qc) if reach else qc
    if distributional:
        out['qc_std'] = ops.constraint_critic_forward(cc, states, actions, sample=True, noise=_NO_TAPE)[1]
    if not reach:
        return out
    a_safe = solver.actor_safe.act(states, eval=True).detach()
    safe_qcs = solver._get_qc(cc(states, a_safe))
    if mlp_multiplier:
        out['lam'] = solver.multiplier(states, safe_qcs)
    return out
