"""Torch-CPU restatement of the reference DRPO hot path (TEST INFRASTRUCTURE ONLY).

Functional restatement over flat ``{state_dict_key: tensor}`` dicts, following
the reference op-for-op so it is bit-exact against the golden fixtures at a
fixed thread count. Every function cites the reference lines it restates
(paths relative to the reference repository root).

Third-party arithmetic restated here (PyTorch 2.10.0, pinned by the fixtures):
torch.optim.Adam single-tensor path, clip_grad_norm_, CosineAnnealingLR,
torch.distributions Normal / TanhTransform / Independent.
"""
import math
import random

import numpy as np
import torch
import torch.nn.functional as F

LOG_SQRT_2PI = math.log(math.sqrt(2 * math.pi))


# ----------------------------------------------------------------------------
# random streams: replay a recorded tape, or draw live in the reference's order
# ----------------------------------------------------------------------------
class TapeRNG:
    """Replays draws recorded by tests/golden/tape.py (kind-checked, in order)."""

    def __init__(self, entries):
        self.entries = list(entries)
        self.pos = 0

    @classmethod
    def from_npz(cls, d, prefix):
        n = int(d[f'{prefix}_n'])
        keys = sorted(k for k in d.files if k.startswith(prefix + '_') and k != f'{prefix}_n')
        assert len(keys) == n, (len(keys), n)
        ents = []
        for k in keys:
            kind = k[len(prefix) + 6:]
            ents.append((kind, d[k]))
        return cls(ents)

    def _next(self, kind, shape=None):
        k, v = self.entries[self.pos]
        assert k == kind, f'tape position {self.pos}: expected {kind}, found {k}'
        if shape is not None:
            assert tuple(v.shape) == tuple(shape), f'tape {kind} shape {v.shape} != {tuple(shape)}'
        self.pos += 1
        return v

    def normal(self, loc, scale):          # torch.normal(loc, scale): eps*scale + loc
        eps = torch.from_numpy(self._next('normal', loc.shape))
        return eps * scale + loc

    def std_normal(self, shape):           # Normal.rsample's _standard_normal (Tensor.normal_)
        return torch.from_numpy(self._next('normal_', shape))

    def randn_like(self, x):
        return torch.from_numpy(self._next('randn_like', x.shape))

    def randint(self, high, n):
        return torch.from_numpy(self._next('randint', (n,)))

    def choice(self, n):                   # random.choice over a length-n sequence -> index
        return int(self._next('choice'))

    def np_choice(self, high, size):       # np.random.choice(high, size, replace=False)
        return self._next('np_choice', (size,))

    def done(self):
        return self.pos == len(self.entries)


class LiveRNG:
    """Draws from the real torch / random / numpy generators with the exact calls the
    reference makes, and records them as a tape (so a HIP run can consume them)."""

    def __init__(self):
        self.entries = []

    def normal(self, loc, scale):
        eps = torch.randn(loc.shape, dtype=loc.dtype)
        self.entries.append(('normal', eps.numpy()))
        return eps * scale + loc

    def std_normal(self, shape):
        eps = torch.empty(shape).normal_()
        self.entries.append(('normal_', eps.numpy()))
        return eps

    def randn_like(self, x):
        eps = torch.randn_like(x)
        self.entries.append(('randn_like', eps.numpy()))
        return eps

    def randint(self, high, n):
        idx = torch.randint(high, [n])
        self.entries.append(('randint', idx.numpy()))
        return idx

    def choice(self, n):
        i = random.choice(range(n))
        self.entries.append(('choice', np.array(i)))
        return i

    def np_choice(self, high, size):
        idx = np.random.choice(high, size=size, replace=False)
        self.entries.append(('np_choice', idx))
        return idx


# ----------------------------------------------------------------------------
# generic MLP pieces (src/torch_util.py:190-211)
# ----------------------------------------------------------------------------
ACTS = {'relu': F.relu, 'tanh': torch.tanh, 'swish': F.silu, 'identity': lambda x: x}


def layer_indices(P, prefix):
    """Indices of the Linear layers of an mlp() Sequential stored under ``prefix``."""
    idx = sorted({int(k[len(prefix):].split('.')[0]) for k in P if k.startswith(prefix) and k.endswith('.weight')})
    return idx


def mlp_forward(P, prefix, x, act='relu', out_act=None, squeeze=False):
    """nn.Sequential from mlp(): Linear, act, ..., Linear [, out_act] [, Squeeze(1)]."""
    a = ACTS[act]
    idx = layer_indices(P, prefix)
    for j, i in enumerate(idx):
        x = F.linear(x, P[f'{prefix}{i}.weight'], P[f'{prefix}{i}.bias'])
        if j < len(idx) - 1:
            x = a(x)
    if out_act is not None:
        x = ACTS[out_act](x)
    if squeeze and x.shape[-1] == 1:
        x = x.squeeze(1)
    return x


# ----------------------------------------------------------------------------
# dynamics ensemble (src/dynamics.py, src/normalization.py)
# ----------------------------------------------------------------------------
def normalize(P, pre, s):
    # src/normalization.py:22-23
    return (s - P[pre + 'state_normalizer.mean']) / (P[pre + 'state_normalizer.std'] + 1e-6)


def _unbatched(P, prefix, x, idx, out_act):
    # src/dynamics.py:258-264 + mlp(activation='swish')
    lids = layer_indices(P, prefix)
    for j, i in enumerate(lids):
        x = F.linear(x, P[f'{prefix}{i}.weight'][idx], P[f'{prefix}{i}.bias'][idx])
        if j < len(lids) - 1 or out_act:
            x = F.silu(x)
    return x


def _batched(P, prefix, x, out_act):
    # BatchedLinear.forward src/dynamics.py:49-52
    lids = layer_indices(P, prefix)
    for j, i in enumerate(lids):
        W, b = P[f'{prefix}{i}.weight'], P[f'{prefix}{i}.bias']
        x = torch.bmm(x, W.transpose(1, 2)) + b.unsqueeze(1)
        if j < len(lids) - 1 or out_act:
            x = F.silu(x)
    return x


def _logvar_clamp(P, pre, lv):
    # src/dynamics.py:120-121
    lv = P[pre + 'max_log_var'] - F.softplus(P[pre + 'max_log_var'] - lv)
    return P[pre + 'min_log_var'] + F.softplus(lv - P[pre + 'min_log_var'])


def ens_forward1(P, pre, s, a, index):
    """BatchedGaussianEnsemble._forward1 (src/dynamics.py:112-122)."""
    x = torch.cat([normalize(P, pre, s), a], dim=-1)
    h = _unbatched(P, pre + 'trunk.', x, index, True)
    diffs = _unbatched(P, pre + 'diff_head.', h, index, False)
    means = diffs + torch.cat([s, torch.zeros([x.shape[0], 1])], dim=1)
    lv = _unbatched(P, pre + 'log_var_head.', h, index, False)
    return means, _logvar_clamp(P, pre, lv)


def ens_forward_all(P, pre, s, a):
    """_forward_all (src/dynamics.py:124-134): s [E,b,S], a [E,b,A]."""
    E, b = s.shape[0], s.shape[1]
    x = torch.cat([normalize(P, pre, s), a], dim=-1)
    h = _batched(P, pre + 'trunk.', x, True)
    diffs = _batched(P, pre + 'diff_head.', h, False)
    means = diffs + torch.cat([s, torch.zeros([E, b, 1])], dim=-1)
    lv = _batched(P, pre + 'log_var_head.', h, False)
    return means, _logvar_clamp(P, pre, lv)


def ens_sample(P, pre, s, a, elite_inds, rng):
    """sample (src/dynamics.py:198-203)."""
    index = elite_inds[rng.choice(len(elite_inds))]
    means, lv = ens_forward1(P, pre, s, a, index)
    stds = torch.exp(lv).sqrt()
    x = means + stds * rng.randn_like(means)
    return x[:, :-1], x[:, -1]


def ens_mse_loss(P, pre, s, a, t):
    """_mse_loss (src/dynamics.py:236-253): per-member heteroscedastic NLL [E]."""
    means, lv = ens_forward_all(P, pre, s, a)
    inv_vars = torch.exp(-lv)
    sq = torch.mean((t - means) ** 2 * inv_vars, dim=(-2, -1))
    return sq + torch.mean(lv, dim=(-2, -1))


def ens_compute_loss(P, pre, s, a, t, E, weight=0.01):
    """compute_loss (src/dynamics.py:143-153) incl. truncation to a multiple of E."""
    n = len(t)
    r = n % E
    if r:
        s, a, t = s[:n - r], a[:n - r], t[:n - r]
    rb = lambda x: x.reshape(E, len(x) // E, *x.shape[1:])
    loss = torch.sum(ens_mse_loss(P, pre, rb(s), rb(a), rb(t)))
    return loss + weight * (P[pre + 'max_log_var'].sum() - P[pre + 'min_log_var'].sum())


def ens_param_keys(P, pre):
    """Optimizer param order (src/dynamics.py:92-101)."""
    keys = []
    for part in ['trunk.', 'diff_head.', 'log_var_head.']:
        for i in layer_indices(P, pre + part):
            keys += [f'{pre}{part}{i}.weight', f'{pre}{part}{i}.bias']
    return keys + [pre + 'min_log_var', pre + 'max_log_var']


def normalizer_fit(X):
    """Normalizer.fit (src/normalization.py:14-19)."""
    mean = X.mean(dim=0)
    std = X.std(dim=0)
    std[std < 1e-6] = 1.0
    return mean, std


def ens_fit(P, pre, opt, buf, steps, E, batch_size, holdout, num_elites, rng, lr=1e-3):
    """fit(steps=...) (src/dynamics.py:155-187). buf: chronological dict of 7 components."""
    states, actions, next_states, rewards = buf['states'], buf['actions'], buf['next_states'], buf['rewards']
    n = len(states)
    P[pre + 'state_normalizer.mean'], P[pre + 'state_normalizer.std'] = normalizer_fit(states)
    targets = torch.cat([next_states, rewards.unsqueeze(1)], dim=1)
    keys = ens_param_keys(P, pre)
    losses = []
    for _ in range(steps):
        idx = rng.randint(n, E * batch_size)
        with torch.enable_grad():
            params = {k: P[k].detach().requires_grad_(True) for k in keys}
            Q = dict(P)
            Q.update(params)
            loss = ens_compute_loss(Q, pre, states[idx], actions[idx], targets[idx], E)
            grads = torch.autograd.grad(loss, [params[k] for k in keys])
        losses.append(loss.item())
        for k, g in zip(keys, grads):
            adam_update(opt, k, P[k], g.clone(), lr, 1e-4)
    hidx = rng.randint(n, holdout).repeat(E, 1)
    with torch.no_grad():
        mse = ens_mse_loss(P, pre, states[hidx], actions[hidx], targets[hidx])
    elites = torch.argsort(mse)[:num_elites].tolist()
    return losses, elites


def ens_fit_epochs(P, pre, opt, buf, epochs, E, batch_size, lr=1e-3):
    """fit(epochs=...) (src/dynamics.py:185-194) -> epochal_training
    (src/train.py:58-100): E * epochs passes of torch.randperm(n) (CPU generator)
    minibatches of E * batch_size rows, the last ragged, one Adam step each; returns
    the per-epoch mean losses."""
    states, actions, next_states, rewards = buf['states'], buf['actions'], buf['next_states'], buf['rewards']
    n = len(states)
    P[pre + 'state_normalizer.mean'], P[pre + 'state_normalizer.std'] = normalizer_fit(states)
    targets = torch.cat([next_states, rewards.unsqueeze(1)], dim=1)
    keys = ens_param_keys(P, pre)
    tb = E * batch_size
    losses = []
    for _ in range(E * epochs):
        perm = torch.randperm(n)
        ep = []
        for bi in range(math.ceil(float(n) / tb)):
            idx = perm[tb * bi:min(tb * (bi + 1), n)]
            with torch.enable_grad():
                params = {k: P[k].detach().requires_grad_(True) for k in keys}
                Q = dict(P)
                Q.update(params)
                loss = ens_compute_loss(Q, pre, states[idx], actions[idx], targets[idx], E)
                grads = torch.autograd.grad(loss, [params[k] for k in keys])
            ep.append(loss.item())
            for k, g in zip(keys, grads):
                adam_update(opt, k, P[k], g.clone(), lr, 1e-4)
        losses.append(float(np.mean(ep)))
    return losses


# ----------------------------------------------------------------------------
# squashed Gaussian policy (src/policy.py:61-100, src/squashed_gaussian.py)
# ----------------------------------------------------------------------------
def policy_params(P, prefix, s, log_std_bounds=(-6, 4)):
    out = mlp_forward(P, prefix, s, 'relu')
    mu, log_std = out.chunk(2, dim=-1)
    lo, hi = log_std_bounds
    log_std = lo + (hi - lo) * torch.sigmoid(log_std)
    std = log_std.exp() * 1.0
    return mu, std


def squashed_log_prob(mu, std, u):
    """Independent(TransformedDistribution(Normal, Tanh)).log_prob at the cached
    pre-tanh value u (torch.distributions; TanhTransform.log_abs_det_jacobian)."""
    ladj = 2.0 * (math.log(2.0) - u - F.softplus(-2.0 * u))
    base = -((u - mu) ** 2) / (2 * std ** 2) - std.log() - LOG_SQRT_2PI
    lp = (0.0 - ladj) + base
    return lp.sum(-1)


def policy_sample(P, prefix, s, rng):
    """distr.sample() (no grad) -> (action, pre-tanh u)."""
    mu, std = policy_params(P, prefix, s)
    u = rng.normal(mu, std)
    return u.tanh(), u, mu, std


def policy_rsample(P, prefix, s, rng):
    mu, std = policy_params(P, prefix, s)
    u = mu + rng.std_normal(mu.shape) * std
    return u.tanh(), u, mu, std


def policy_mean(P, prefix, s):
    mu, _ = policy_params(P, prefix, s)
    return torch.tanh(mu)


# ----------------------------------------------------------------------------
# batched env constraint functions (numpy, reference numerics)
# ----------------------------------------------------------------------------
QUAD_X_THRESHOLD = 2.0    # safe_control_gym Quadrotor.x_threshold: PARITY UNPINNED
QUAD_Z_THRESHOLD = 3.0    # safe_control_gym Quadrotor.z_threshold: PARITY UNPINNED


def constraints_point_robot(s):
    """src/env/point_robot.py:96-131."""
    hazards = [np.array([0.4, -1.2]), np.array([-0.4, 1.2])]
    min_dist = np.full(s.shape[0], float('inf'))
    for hp in hazards:
        min_dist = np.minimum(np.linalg.norm(hp[:2] - s[:, :2], axis=1), min_dist)
    h = 0.8 - min_dist
    oob = np.logical_or(np.logical_or(s[:, 0] < -3.0, s[:, 0] > 3.0),
                        np.logical_or(s[:, 1] < -3.0, s[:, 1] > 3.0))
    goal = np.linalg.norm(s[:, :2] - np.array([2.2, 2.2]), axis=1) <= 0.3
    return np.logical_or(oob, goal), h > 0, h[:, None]


def _bounded(s, dims, lb, ub):
    """BoundedConstraint.get_value (src/env/poles/constraints.py:89-105,216-247): [-x+lb, x-ub]."""
    x = s[:, dims].astype(np.float64)
    return np.concatenate([-x + np.asarray(lb, np.float64), x - np.asarray(ub, np.float64)], axis=1)


def constraints_quadrotor(s):
    """src/env/quadrotor/quadrotor.py:83-158 (bounds from constrained_tracking_reset.yaml)."""
    h = _bounded(s, [2], [0.5], [1.5])
    viol = np.any(h > 0.0, axis=-1)
    th = np.float32(85 * math.pi / 180)
    x, z, theta = s[:, 0], s[:, 2], s[:, 4]
    xt, zt = np.float32(QUAD_X_THRESHOLD), np.float32(QUAD_Z_THRESHOLD)
    done = (x < -xt) | (x > xt) | (z < -zt) | (z > zt) | (theta < -th) | (theta > th)
    return np.logical_or(done, viol), viol, h


def constraints_cartpole(s):
    """src/env/poles/inverted_pendulum.py:79-121 (+ constraints.py BoundedConstraint)."""
    h = _bounded(s, [0, 1], [-0.9, -0.2], [0.9, 0.2])
    v = np.any(h > 0.0, axis=-1)
    return v, v, h


def constraints_tracking(s, surr_start=47, n_surr=1, veh_length=4.8, veh_width=2.0):
    """src/env/tracking/pyth_veh3dofconti_surrcstr_data.py:253-338 (float32 geometry,
    float64 final 2r - min_dist as in the reference)."""
    s = s.astype(np.float32)
    err_done = np.logical_or(np.logical_or(np.abs(s[:, 0]) > 5, np.abs(s[:, 1]) > 2), np.abs(s[:, 2]) > np.pi)
    d = (veh_length - veh_width) / 2
    r = np.sqrt(2) / 2 * veh_width
    ego = np.array([[d, 0], [-d, 0]], dtype=np.float32)
    c, sn = np.cos(s[:, 6])[:, None], np.sin(s[:, 6])[:, None]
    surr = s[:, surr_start:].reshape(-1, n_surr, 4)
    xs, ys, ph = surr[:, :, 0], surr[:, :, 1], surr[:, :, 2]
    xe = xs * c + ys * sn
    ye = -xs * sn + ys * c
    centers = np.stack((np.stack((xe + d * np.cos(ph), ye + d * np.sin(ph)), axis=2),
                        np.stack((xe - d * np.cos(ph), ye - d * np.sin(ph)), axis=2)), axis=2)
    ego = ego[np.newaxis, np.newaxis, ...]
    ds = [np.linalg.norm(ego[..., i, :] - centers[..., j, :], axis=-1) for i in (0, 1) for j in (0, 1)]
    min_dist = np.min(np.min(np.stack(ds, axis=1), axis=-1), axis=-1)
    h = 2 * r - min_dist
    return err_done, h > 0, np.asarray(h, np.float64)[:, None]


ENV_CONSTRAINTS = {'point-robot': constraints_point_robot, 'quadrotor': constraints_quadrotor,
                   'cartpole': constraints_cartpole, 'tracking': constraints_tracking}


def env_fns(env):
    """(done, violation, constraint_value) as the reference's torchify'd lambdas
    (src/smbpo.py:63-65): bool, bool, float32 [n] (C == 1) or [n, C]."""
    f = ENV_CONSTRAINTS[env]

    def run(s):
        dn, v, h = f(s.detach().numpy())
        h = torch.from_numpy(np.asarray(h)).float()
        if h.shape[1] == 1:
            h = h[:, 0]
        return torch.from_numpy(np.asarray(dn)), torch.from_numpy(np.asarray(v)), h
    return run


# ----------------------------------------------------------------------------
# SMBPO.rollout (src/smbpo.py:229-249, src/torch_util.py:41-48)
# ----------------------------------------------------------------------------
COMPONENTS = ('states', 'actions', 'next_states', 'rewards', 'dones', 'violations', 'constraint_values')


@torch.no_grad()
def rollout(P, actor_pre, model_pre, elite_inds, replay_states, env, B, H, rng):
    """Returns the rows written to the virtual buffer, in order (dict of 7 tensors)."""
    fns = env_fns(env)
    idx = torch.from_numpy(np.asarray(rng.np_choice(replay_states.shape[0], B)))
    states = replay_states.index_select(0, idx)
    rows = {k: [] for k in COMPONENTS}
    for _ in range(H):
        actions, _, _, _ = policy_sample(P, actor_pre, states, rng)
        next_states, rewards = ens_sample(P, model_pre, states, actions, elite_inds, rng)
        dones, viols, h = fns(next_states)
        for k, v in zip(COMPONENTS, (states, actions, next_states, rewards, dones, viols, h)):
            rows[k].append(v)
        cont = ~dones
        if cont.sum() == 0:
            break
        states = next_states[cont]
    return {k: torch.cat(v) for k, v in rows.items()}


# ----------------------------------------------------------------------------
# optimisation primitives (torch.optim.Adam single-tensor path, clip_grad_norm_,
# CosineAnnealingLR, update_ema src/torch_util.py:223-226)
# ----------------------------------------------------------------------------
def adam_update(opt, key, param, grad, lr, weight_decay, betas=(0.9, 0.999), eps=1e-8):
    st = opt.setdefault(key, {'step': 0, 'm': torch.zeros_like(param), 'v': torch.zeros_like(param)})
    st['step'] += 1
    if weight_decay != 0:
        grad = grad.add(param, alpha=weight_decay)
    st['g'] = grad       # tests: the effective (clipped + L2) gradient of this step
    st['m'].lerp_(grad, 1 - betas[0])
    st['v'].mul_(betas[1]).addcmul_(grad, grad, value=1 - betas[1])
    step = float(st['step'])
    bc1 = 1 - betas[0] ** step
    bc2 = 1 - betas[1] ** step
    denom = (st['v'].sqrt() / (bc2 ** 0.5)).add_(eps)
    param.addcdiv_(st['m'], denom, value=-(lr / bc1))


def clip_grads(grads, max_norm):
    norms = [torch.linalg.vector_norm(g, 2.0) for g in grads]
    total = torch.linalg.vector_norm(torch.stack(norms), 2.0)
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    for g in grads:
        g.mul_(coef)
    return total


class Cosine:
    """CosineAnnealingLR (recursive form, torch 2.10)."""

    def __init__(self, base_lr, T_max, eta_min):
        self.base, self.T, self.eta = base_lr, T_max, eta_min
        self.lr = base_lr
        self.last_epoch = 0

    def step(self):
        self.last_epoch += 1
        e, T = self.last_epoch, self.T
        if (e - 1 - T) % (2 * T) == 0:
            self.lr = self.lr + (self.base - self.eta) * (1 - math.cos(math.pi / T)) / 2
        else:
            self.lr = (1 + math.cos(math.pi * e / T)) / (1 + math.cos(math.pi * (e - 1) / T)) * \
                (self.lr - self.eta) + self.eta


def ema(P, target_pre, source_pre, rate):
    for k in [k for k in P if k.startswith(source_pre)]:
        tk = target_pre + k[len(source_pre):]
        P[tk] = rate * P[k] + (1 - rate) * P[tk]


# ----------------------------------------------------------------------------
# SSAC networks (src/ssac.py:17-111)
# ----------------------------------------------------------------------------
def critic_all(P, pre, s, a):
    sa = torch.cat([s, a], -1)
    n = len({k[len(pre) + 3:].split('.')[0] for k in P if k.startswith(pre + 'qs.')})
    return [mlp_forward(P, f'{pre}qs.{i}.', sa, 'relu', squeeze=True) for i in range(n)]


def cons_critic(P, pre, s, a, mode='mean', std_ratio=2.0, rng=None, lmin=-4.0, lmax=4.0):
    """ConstraintCritic.forward (src/ssac.py:64-92). mode: mean | uncertainty | sample."""
    sa = torch.cat([s, a], -1)
    h = mlp_forward(P, pre + 'trunk.', sa, 'relu', out_act='relu')
    mean = mlp_forward(P, pre + 'mean_head.', h, 'relu', squeeze=True)
    if mode == 'mean':
        return mean
    ls = mlp_forward(P, pre + 'log_std_head.', h, 'relu', squeeze=True)
    ls = lmax - F.softplus(lmax - ls)
    ls = lmin + F.softplus(ls - lmin)
    std = ls.exp()
    noise = rng.randn_like(std)
    if mode == 'uncertainty':
        return mean + torch.mul(std_ratio, std)
    noise = torch.clamp(noise, -2., 2.)
    return mean, std, mean + torch.mul(noise, std)


def multiplier(P, pre, s, qc, ub=50.0):
    x = mlp_forward(P, pre + 'lam.', torch.cat([s, qc.unsqueeze(-1)], -1), 'tanh', squeeze=True)
    return ub / 2. * (1. + torch.tanh(x / ub * 2))


def get_qc(qc, C):
    return torch.max(qc, dim=-1)[0] if C > 1 else qc


# ----------------------------------------------------------------------------
# SSAC updates (src/ssac.py:284-578) on a flat state dict
# ----------------------------------------------------------------------------
class SSACOracle:
    GROUPS = {'critic': ['critic.', 'constraint_critic.'], 'actor': ['actor.'],
              'actor_safe': ['actor_safe.'], 'multiplier': ['multiplier.']}

    def __init__(self, P, cfg, C, A):
        """P: solver-relative state dict (keys 'actor.net.0.weight', ...). cfg: dict."""
        self.P = {k: v.clone().float() for k, v in P.items()}
        self.log_alpha = torch.tensor(float(self.P.pop('log_alpha', torch.tensor(math.log(cfg.get('init_alpha', 1.0))))))
        self.c = dict(discount=0.99, tau=0.005, grad_norm=5.0, std_ratio=2.0, ub=50.0, lam_epsilon=1.0,
                      penalty_lb=-1.0, penalty_ub=100.0, constraint_threshold=0.0, qc_td_bound=5.0,
                      critic_lr=3e-4, critic_lr_end=8e-5, actor_lr=8e-5, actor_lr_end=4e-5,
                      multiplier_lr=3e-4, multiplier_lr_end=1e-5, distributional=True, uncertainty=True,
                      deterministic_backup=False, target_entropy=-float(A), batch_size=256,
                      updates_per_training=1000, actor_update_interval=2, multiplier_update_interval=5,
                      mlp_multiplier=True, fixed_multiplier=15.0, autotune_alpha=True, use_log_alpha_loss=False,
                      cost=False)
        self.c.update(cfg)
        if self.c.get('constrained_fcn') == 'cost':
            self.c['cost'] = True
        # the cost certificate is one value per row (src/ssac.py:191)
        self.C, self.A = (1 if self.c['cost'] else C), A
        c = self.c
        T = c['updates_per_training']
        self.opt = {g: {} for g in ['critic', 'actor', 'actor_safe', 'multiplier', 'alpha']}
        self.sched = {'critic': Cosine(c['critic_lr'], T, c['critic_lr_end']),
                      'actor': Cosine(c['actor_lr'], int(T / c['actor_update_interval']), c['actor_lr_end']),
                      'actor_safe': Cosine(c['actor_lr'], int(T / c['actor_update_interval']), c['actor_lr_end']),
                      'multiplier': Cosine(c['multiplier_lr'], int(T / c['multiplier_update_interval']),
                                           c['multiplier_lr_end'])}

    def keys(self, prefixes):
        return [k for k in self.P for p in prefixes if k.startswith(p)]

    def _grad(self, loss_fn, keys):
        with torch.enable_grad():
            params = {k: self.P[k].detach().requires_grad_(True) for k in keys}
            Q = dict(self.P)
            Q.update(params)
            loss = loss_fn(Q)
            grads = torch.autograd.grad(loss, [params[k] for k in keys], allow_unused=True)
        # params outside the graph keep grad=None: torch's clip and Adam skip them
        out = {k: g.clone() for k, g in zip(keys, grads) if g is not None}
        self.last_grads = getattr(self, 'last_grads', {})
        self.last_grads.update(out)      # tests: conditioning of each element's Adam step
        return loss.detach(), out

    @property
    def alpha(self):
        return self.log_alpha.exp()

    # --- src/ssac.py:284-294
    def compute_target(self, s2, r, d, rng):
        with torch.no_grad():
            a2, u, mu, std = policy_sample(self.P, 'actor.net.', s2, rng)
            logp = squashed_log_prob(mu, std, u)
            nv = torch.min(*critic_all(self.P, 'critic_target.', s2, a2))
            if not self.c['deterministic_backup']:
                nv = nv - self.alpha.detach() * logp
            return r + self.c['discount'] * (1. - d.float()) * nv

    # --- src/ssac.py:304-413 (reachability; distributional or vanilla; or the cost certificate)
    def compute_cons_target(self, s, a, s2, d, h, rng, P=None, v=None):
        P = self.P if P is None else P
        g, C = self.c['discount'], self.C
        with torch.no_grad():
            if self.c['cost']:
                # src/ssac.py:306-310: a' ~ pi(s'), Qc_target(s', a'), one-step violation cost
                a2, _, _, _ = policy_sample(P, 'actor.net.', s2, rng)
                q2 = cons_critic(P, 'constraint_critic_target.', s2, a2, 'mean')
                return v.float() + g * (1. - d.float()) * q2, None
            robust = self.c['uncertainty'] and not self.c['distributional']
            if not robust:
                a2, _, _, _ = policy_sample(P, 'actor_safe.net.', s2, rng)
            dones = d.tile((C, 1)).t().squeeze().float()
            if self.c['uncertainty'] and self.c['distributional']:
                _, _, q2 = cons_critic(P, 'constraint_critic_target.', s2, a2, 'sample', self.c['std_ratio'], rng)
                qm = cons_critic(P, 'constraint_critic.', s, a, 'mean')
                nonterm = (1. - g) * h + g * torch.maximum(h, q2)
                y = nonterm * (1 - dones) + h * dones
                diff = torch.clamp(y - qm, min=-self.c['qc_td_bound'], max=self.c['qc_td_bound'])
                return y, diff + qm
            if self.c['uncertainty']:
                # robust: s' from one elite member of the dynamics model, done from the
                # env's check_done on it (src/ssac.py:387-400)
                s2m, _ = ens_sample(P, 'model_ensemble.', s, a, self.c['elites'], rng)
                dm, _, _ = env_fns(self.c['env'])(s2m)
                a2m, _, _, _ = policy_sample(P, 'actor_safe.net.', s2m, rng)
                q2 = cons_critic(P, 'constraint_critic_target.', s2m, a2m, 'mean')
                dones = dm.tile((C, 1)).t().squeeze()
                nonterm = (1. - g) * h + g * torch.maximum(h, q2)
                return torch.where(dones, h, nonterm), None
            q2 = cons_critic(P, 'constraint_critic_target.', s2, a2, 'mean')
            nonterm = (1. - g) * h + g * torch.maximum(h, q2)
            return nonterm * (1 - dones.float()) + h * dones.float(), None

    def update_critic(self, s, a, s2, r, d, v, h, rng):
        """src/ssac.py:437-456."""
        y = self.compute_target(s2, r, d, rng)
        yc, yb = self.compute_cons_target(s, a, s2, d, h, rng, v=v)
        dist = self.c['distributional']
        rs = rng

        def loss_fn(Q):
            qs = critic_all(Q, 'critic.', s, a)
            lq = sum([F.mse_loss(q, y) for q in qs]) / len(qs)
            mu, sd, _ = cons_critic(Q, 'constraint_critic.', s, a, 'sample', self.c['std_ratio'], rs)
            if dist:
                lqc = torch.mean(torch.pow(mu - yc, 2) / (2 * torch.pow(sd.detach(), 2)) +
                                 torch.pow(mu.detach() - yb, 2) / (2 * torch.pow(sd, 2)) + torch.log(sd))
            else:
                lqc = F.mse_loss(mu, yc)
            self._last = (lq.detach(), lqc.detach())
            return lq + lqc

        kc = self.keys(['critic.'])
        kcc = self.keys(['constraint_critic.'])
        _, grads = self._grad(loss_fn, kc + kcc)
        clip_grads([grads[k] for k in kc if k in grads], self.c['grad_norm'])
        clip_grads([grads[k] for k in kcc if k in grads], self.c['grad_norm'])
        lr = self.sched['critic'].lr
        for k in [k for k in kc + kcc if k in grads]:
            adam_update(self.opt['critic'], k, self.P[k], grads[k], lr, 1e-4)
        self.sched['critic'].step()
        tau = self.c['tau']
        ema(self.P, 'critic_target.', 'critic.', tau)
        ema(self.P, 'constraint_critic_target.', 'constraint_critic.', tau)
        return self._last

    def update_actor_and_alpha(self, s, rng):
        """src/ssac.py:458-527 (reachability; MLP or scalar multiplier; alpha flags)."""
        C, sr = self.C, self.c['std_ratio']
        dist = self.c['distributional']
        mlp_mult = self.c['mlp_multiplier']
        mode = 'uncertainty' if dist else 'mean'
        store = {}

        def actor_loss(Q):
            a, u, mu, std = policy_rsample(Q, 'actor.net.', s, rng)
            logp = squashed_log_prob(mu, std, u)
            qs_i = rng.choice(2)
            sa_q = mlp_forward(Q, f'critic.qs.{qs_i}.', torch.cat([s, a], -1), 'relu', squeeze=True)
            alpha = self.alpha
            unc = torch.mean(alpha.detach() * logp - sa_q)
            aqc = get_qc(cons_critic(Q, 'constraint_critic.', s, a, mode, sr, rng), C)
            if mlp_mult:
                with torch.no_grad():
                    a_safe = policy_mean(Q, 'actor_safe.net.', s)
                    sqc = get_qc(cons_critic(Q, 'constraint_critic.', s, a_safe, mode, sr, rng), C)
                    lams = multiplier(Q, 'multiplier.', s, sqc, self.c['ub'])
            else:   # src/ssac.py:480-483
                lams = self.c['fixed_multiplier']
                aqc = torch.clamp(aqc, min=self.c['penalty_lb'], max=self.c['penalty_ub'])
            store['logp'] = logp.detach()
            return unc + torch.mean(torch.mul(lams, aqc))

        ka = self.keys(['actor.'])
        _, ga = self._grad(actor_loss, ka)
        # safe actor loss draws after the actor loss (src/ssac.py:488-494); the cost
        # certificate has none (optimizers [actor, alpha], src/ssac.py:509-513)
        kas = [] if self.c['cost'] else self.keys(['actor_safe.'])

        def safe_loss(Q):
            a_s, _, _, _ = policy_rsample(Q, 'actor_safe.net.', s, rng)
            return torch.mean(get_qc(cons_critic(Q, 'constraint_critic.', s, a_s, mode, sr, rng), C))

        # alpha loss (src/ssac.py:498-501); uses log_prob.detach(); the coefficient is
        # alpha, or log_alpha itself with use_log_alpha_loss
        coef = 1.0 if self.c['use_log_alpha_loss'] else self.alpha
        alpha_grad = -coef * torch.mean(store['logp'] + self.c['target_entropy'])
        gs = self._grad(safe_loss, kas)[1] if kas else {}
        clip_grads([ga[k] for k in ka], self.c['grad_norm'])
        lr = self.sched['actor'].lr
        for k in ka:
            adam_update(self.opt['actor'], k, self.P[k], ga[k], lr, 1e-4)
        self.sched['actor'].step()
        auto = self.c['autotune_alpha']
        if auto:
            la = self.log_alpha.clone()
            adam_update(self.opt['alpha'], 'log_alpha', la, torch.as_tensor(alpha_grad).detach().clone(),
                        self.c['actor_lr'], 0)
            self.log_alpha = la
        # the reference clips / schedules the safe actor at optimizer index 2, which is
        # the safe actor only when the alpha optimizer sits at index 1 (src/ssac.py:515-527)
        if auto and kas:
            clip_grads([gs[k] for k in kas], self.c['grad_norm'])
        lr = self.sched['actor_safe'].lr
        for k in kas:
            adam_update(self.opt['actor_safe'], k, self.P[k], gs[k], lr, 1e-4)
        if auto and kas:
            self.sched['actor_safe'].step()

    def update_multiplier(self, s, rng):
        """src/ssac.py:529-578 (MLP or scalar multiplier)."""
        C, sr = self.C, self.c['std_ratio']
        mode = 'uncertainty' if self.c['distributional'] else 'mean'
        with torch.no_grad():
            a, _, _, _ = policy_rsample(self.P, 'actor.net.', s, rng)
            aqc = get_qc(cons_critic(self.P, 'constraint_critic.', s, a, mode, sr, rng), C)
            pen = torch.clamp(aqc - self.c['constraint_threshold'], min=self.c['penalty_lb'], max=self.c['penalty_ub'])
        if not self.c['mlp_multiplier']:
            # lam_loss = -mean(softplus(m) * penalty): plain Adam (lr multiplier_lr, no
            # weight decay), no clip, no schedule (src/ssac.py:564-578)
            _, gm = self._grad(lambda Q: -torch.mean(torch.mul(F.softplus(Q['multiplier']), pen)), ['multiplier'])
            adam_update(self.opt['multiplier'], 'multiplier', self.P['multiplier'], gm['multiplier'],
                        self.c['multiplier_lr'], 0)
            return
        with torch.no_grad():
            a_safe = policy_mean(self.P, 'actor_safe.net.', s)
            sqc = get_qc(cons_critic(self.P, 'constraint_critic.', s, a_safe, mode, sr, rng), C)
        ub, le = self.c['ub'], self.c['lam_epsilon']

        def loss_fn(Q):
            lams = multiplier(Q, 'multiplier.', s, sqc, ub)
            ls, lu = torch.mul(sqc <= 0, lams), torch.mul(sqc > 0, lams)
            return -0.5 * torch.mean(torch.mul(ls, pen.detach())) + F.mse_loss(lu, (sqc > 0) * (ub - le))

        km = self.keys(['multiplier.'])
        _, gm = self._grad(loss_fn, km)
        clip_grads([gm[k] for k in km], self.c['grad_norm'])
        lr = self.sched['multiplier'].lr
        for k in km:
            adam_update(self.opt['multiplier'], k, self.P[k], gm[k], lr, 1e-4)
        self.sched['multiplier'].step()


def preprocess_batch(samples, reward_scale, alive_bonus, constraint_scale, constraint_offset):
    """SMBPO.update_solver reward / constraint preprocessing (src/smbpo.py:260-270)."""
    s = list(samples)
    if reward_scale != 0:
        s[3] = s[3] * reward_scale
    if alive_bonus != 0:
        s[3] = s[3] + alive_bonus
    s[6] = s[6] * constraint_scale
    s[6] = s[6] + (s[6] > 0).float() * constraint_offset
    return s


# ----------------------------------------------------------------------------
# circular sample buffer (src/sampling.py:12-151,215-251) and the SMBPO loop
# pieces that sit on the hot path (src/smbpo.py:214-291)
# ----------------------------------------------------------------------------
class RingBuffer:
    def __init__(self, S, A, C, capacity):
        self.capacity = capacity
        self.ptr = 0
        shapes = {'states': [S], 'actions': [A], 'next_states': [S], 'rewards': [], 'dones': [],
                  'violations': [], 'constraint_values': [] if C == 1 else [C]}
        dt = {'dones': torch.bool, 'violations': torch.bool}
        self.bufs = {k: torch.zeros([capacity, *shp], dtype=dt.get(k, torch.float)) for k, shp in shapes.items()}

    def __len__(self):
        return min(self.ptr, self.capacity)

    def extend(self, rows):
        n = len(rows['states'])
        assert n <= self.capacity
        i = self.ptr % self.capacity
        end = i + n
        for k, buf in self.bufs.items():
            if end <= self.capacity:
                buf[i:end] = rows[k]
            else:
                fit = self.capacity - i
                buf[-fit:] = rows[k][:fit]
                buf[:end - self.capacity] = rows[k][-(end - self.capacity):]
        self.ptr += n

    def get(self, name):
        buf = self.bufs[name]
        if self.ptr <= self.capacity:
            return buf[:self.ptr]
        i = self.ptr % self.capacity
        return torch.cat([buf[i:], buf[:i]])

    def sample(self, n, rng):
        idx = rng.randint(len(self), n)
        return [self.bufs[k][idx] for k in COMPONENTS]


class SMBPOOracle:
    """Hot-path slice of SMBPO: update_models, rollout, update_solver, rollout_and_update."""

    def __init__(self, sd, env, cfg, S, A, C):
        """sd: full SMBPO state dict ('solver.*', 'model_ensemble.*'); cfg: dict of SMBPO fields."""
        self.c = cfg
        self.env, self.S, self.A, self.C = env, S, A, C
        self.M = {k: v.clone() for k, v in sd.items() if k.startswith('model_ensemble.')}
        solver = {k[len('solver.'):]: v for k, v in sd.items()
                  if k.startswith('solver.') and not k.startswith('solver.model_ensemble.')}
        self.ssac = SSACOracle(solver, cfg['sac'], C, A)
        self.model_opt = {}
        self.elite_inds = None
        self.replay = RingBuffer(S, A, C, cfg['buffer_max'])
        self.virt = RingBuffer(S, A, C, cfg['buffer_max'])
        self.critic_losses, self.cons_losses = [], []

    def update_models(self, steps, rng):
        m = self.c['model']
        buf = {k: self.replay.get(k) for k in COMPONENTS}
        losses, self.elite_inds = ens_fit(self.M, 'model_ensemble.', self.model_opt, buf, steps, m['E'],
                                          m['batch_size'], m['holdout'], m['num_elites'], rng)
        return losses

    def rollout(self, rng):
        P = dict(self.M)
        P.update({'actor.' + k[len('actor.'):]: v for k, v in self.ssac.P.items() if k.startswith('actor.')})
        rows = rollout(P, 'actor.net.', 'model_ensemble.', self.elite_inds, self.replay.get('states'),
                       self.env, self.c['B'], self.c['H'], rng)
        self.virt.extend(rows)
        return rows

    def update_solver(self, rng, update_actor=True, update_multiplier=False):
        B = self.c['sac']['batch_size']
        n_real = int(self.c['real_fraction'] * B)
        real = self.replay.sample(n_real, rng)
        virt = self.virt.sample(B - n_real, rng)
        batch = [torch.cat([r, v]) for r, v in zip(real, virt)]
        batch = preprocess_batch(batch, self.c['reward_scale'], self.c['alive_bonus'],
                                 self.c['constraint_scale'], self.c['constraint_offset'])
        lq, lqc = self.ssac.update_critic(*batch, rng)
        self.critic_losses.append(lq)
        self.cons_losses.append(lqc)
        if update_actor:
            self.ssac.update_actor_and_alpha(batch[0], rng)
        if update_multiplier:
            self.ssac.update_multiplier(batch[0], rng)

    def rollout_and_update(self, rng):
        self.rollout(rng)
        sc = self.ssac.c
        for step in range(self.c['solver_updates_per_step']):
            self.update_solver(rng, update_actor=step % sc['actor_update_interval'] == 0,
                               update_multiplier=step % sc['multiplier_update_interval'] == 0)
