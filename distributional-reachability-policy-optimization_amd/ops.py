"""Host glue: turns the reference-API calls into C-ABI launches (libdrpo_hip.so).

Everything here only marshals pointers, shapes and noise; all arithmetic runs in
the HIP kernels. No CPU fallback: a missing library or non-device tensors raise.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._abi import RolloutDesc


def _dev(x, device, dtype=None):
    t = torch.as_tensor(x, device=device)
    return t if dtype is None else t.to(dtype)


# ---------------------------------------------------------------------------
# rollout (src/smbpo.py:229-249)
# ---------------------------------------------------------------------------
def _tape_rollout_noise(noise, H, B, A, S1):
    """Parity mode: pull the reference's rollout draws from the tape. Returns
    (init_idx, members, eps_a [H,B,A], eps_m [H,B,S1], per-step row counts)."""
    eps_a = np.zeros((H, B, A), np.float32)
    eps_m = np.zeros((H, B, S1), np.float32)
    ks, ns = [], []
    for t in range(H):
        if noise.peek() != 'normal':
            break
        ea = noise._take('normal')
        k = noise.choice(None)
        em = noise._take('randn_like')
        n = ea.shape[0]
        assert em.shape == (n, S1) and ea.shape == (n, A)
        eps_a[t, :n], eps_m[t, :n] = ea, em
        ks.append(k)
        ns.append(n)
    return ks, ns, eps_a, eps_m


class EventTimer:
    """Pool of HIP events recorded by the library around its dominant kernels."""

    def __init__(self, n):
        L = _lib.lib()
        self.events = (ctypes.c_void_p * n)()
        for i in range(n):
            ev = ctypes.c_void_p()
            _lib.check(L.drpo_event_create(ctypes.byref(ev)), 'event_create')
            self.events[i] = ev
        self.n = n

    def elapsed_pairs(self, npairs):
        """ms between events (2i, 2i+1) for i < npairs (call after synchronize)."""
        L = _lib.lib()
        out = []
        for i in range(npairs):
            ms = ctypes.c_float()
            _lib.check(L.drpo_event_elapsed_ms(ctypes.byref(ms), self.events[2 * i], self.events[2 * i + 1]), 'elapsed')
            out.append(ms.value)
        return out


_VB_FIELDS = ('_states', '_actions', '_next_states', '_rewards', '_constraint_values', '_dones', '_violations',
              '_pointer')
_ROLLOUT_CACHE_MAX = 8


def _rollout_static(alg, policy, B, H):
    """The per-(shapes, parameter groups, buffers) part of the rollout descriptor: the
    packed-mirror and bias pointers, env parameters, normalizer / log-var bound and
    virtual-buffer pointers, and the workspace. Built once and cached on ``alg``; per
    call only the members, the noise, the initial-state source and the events change.
    (Building it took ~20 tensor views per call: most of the call's host time.)"""
    model = alg.model_ensemble
    vb = alg.virt_buffer._module
    pg, mg = policy.group, model.group
    norm = model.state_normalizer
    # every device pointer the descriptor stores is part of the key (a buffer reallocated
    # under one of them must never leave a stale pointer behind)
    key = (id(policy), B, H, pg.data.data_ptr(), pg.packed.data_ptr(), mg.data.data_ptr(), mg.packed.data_ptr(),
           norm.mean.data_ptr(), norm.std.data_ptr(), model.min_log_var.data_ptr(), model.max_log_var.data_ptr(),
           vb.capacity) + tuple(getattr(vb, f).data_ptr() for f in _VB_FIELDS)
    cache = alg.__dict__.setdefault('_rollout_desc_cache', {})
    hit = cache.get(key)
    if hit is not None:
        return hit
    if len(cache) >= _ROLLOUT_CACHE_MAX:   # (B, H) or buffers changed: drop the old entries
        cache.clear()
    L = _lib.lib()
    S, A, C = alg.state_dim, alg.action_dim, alg.con_dim
    pa = [(pg.pview(f'net.{2 * i}.weight')[0], pg.view(f'net.{2 * i}.bias')) for i in range(policy.spec.n_layers)]

    def mviews(prefix, spec):   # packed mirrors of member 0 (the kernel adds member * packed size)
        return [(mg.pview(f'{prefix}{2 * i}.weight')[0], mg.view(f'{prefix}{2 * i}.bias'))
                for i in range(spec.n_layers)]
    trunk, diff, logv = (mviews('trunk.', model.trunk_spec), mviews('diff_head.', model.diff_spec),
                         mviews('log_var_head.', model.logvar_spec))
    ep = alg.env_params
    d = RolloutDesc()
    d.S, d.A, d.C, d.Ha, d.Hm, d.B, d.H = S, A, C, policy.spec.dims[1], model.hidden_dim, B, H
    d.env_id, d.tracking_surr_start, d.tracking_n_surr = ep['env_id'], ep['tracking_surr_start'], ep['tracking_n_surr']
    d.env_thr0, d.env_thr1 = ep['thr0'], ep['thr1']
    (d.aW1, d.ab1), (d.aW2, d.ab2), (d.aW3, d.ab3) = [(W.data_ptr(), b.data_ptr()) for W, b in pa]
    (d.mW1, d.mb1), (d.mW2, d.mb2) = [(W.data_ptr(), b.data_ptr()) for W, b in trunk]
    (d.dW1, d.db1), (d.dW2, d.db2) = [(W.data_ptr(), b.data_ptr()) for W, b in diff]
    (d.lW1, d.lb1), (d.lW2, d.lb2) = [(W.data_ptr(), b.data_ptr()) for W, b in logv]
    d.norm_mean, d.norm_std = norm.mean.data_ptr(), norm.std.data_ptr()
    d.min_lv, d.max_lv = model.min_log_var.data_ptr(), model.max_log_var.data_ptr()
    d.vs, d.va, d.vs2, d.vr = vb._states.data_ptr(), vb._actions.data_ptr(), vb._next_states.data_ptr(), \
        vb._rewards.data_ptr()
    d.vh, d.vd, d.vv = vb._constraint_values.data_ptr(), vb._dones.data_ptr(), vb._violations.data_ptr()
    d.vptr, d.vcap = vb._pointer.data_ptr(), vb.capacity
    # a workspace of its own per entry (the cached pointers must never see it reallocated)
    ws = alg._workspace(f'rollout.{B}.{H}', L.drpo_rollout_workspace_size(B, S, H))
    d.workspace = ws.data_ptr()
    members = (ctypes.c_int * H)()
    d.members = members
    off = L.drpo_rollout_count_offset(B, S, H)
    count = ws[off:off + 8].view(torch.int64)[0]
    hit = cache[key] = (d, members, count)
    return hit


def rollout(alg, policy, initial_states, noise, timer=None, eps_layout=0):
    """One imagined rollout (src/smbpo.py:229-249) into alg.virt_buffer.

    Engine (``alg.rollout_engine``, 0 = auto): 2 = fused horizon kernel (default for
    device noise), 1 = one launch per horizon step (used for recorded reference
    draws, which are indexed by the compacted row of each step). ``eps_layout=1``
    marks a tape whose per-step draws are indexed by the original batch row
    ([B] rows every step), which drives engine 2 with recorded draws."""
    L = _lib.lib()
    dev = alg.device
    B, H = alg.rollout_batch_size, alg.horizon
    S, A = alg.state_dim, alg.action_dim
    model = alg.model_ensemble
    rb, vb = alg.replay_buffer._module, alg.virt_buffer._module
    _lib.require_device(policy.group.data, model.group.data, vb._states)

    # initial states: chronological replay indices (np.random.choice without replacement)
    if initial_states is not None:
        # the reference rolls out exactly len(initial_states) rows (src/smbpo.py:230-233)
        src = initial_states.contiguous().float()
        _lib.require_device(src)
        B = len(src)
        src_ptr = src_cap = B
        init_idx = torch.arange(B, device=dev, dtype=torch.int64)
    else:
        src, src_ptr, src_cap = rb._states, rb.pointer, rb.capacity
        n_real = min(src_ptr, src_cap)
        idx = noise.np_choice(n_real, B)
        init_idx = None if idx is None else _dev(idx, dev, torch.int64)

    assert B * H <= vb.capacity, 'We do not support extending by more than buffer capacity'
    S1 = S + 1
    if noise.parity:
        ks, ns, eps_a, eps_m = _tape_rollout_noise(noise, H, B, A, S1)
        members = [model._elite_inds[k] for k in ks] + [0] * (H - len(ks))
        eps_a_t, eps_m_t = _dev(eps_a, dev), _dev(eps_m, dev)
    else:
        ns = None
        elites = model._elite_inds
        members = [elites[noise.choice(len(elites))] for _ in range(H)]
        eps_a_t = eps_m_t = None
    ctr = noise.next()

    start_ptr = vb.pointer if vb._host_ptr is not None else None
    policy.group.ensure_packed()
    model.group.ensure_packed()
    d, marr, count = _rollout_static(alg, policy, B, H)
    marr[:] = members
    d.replay_states, d.replay_ptr, d.replay_cap = src.data_ptr(), src_ptr, src_cap
    d.init_idx = 0 if init_idx is None else init_idx.data_ptr()
    d.eps_a = 0 if eps_a_t is None else eps_a_t.data_ptr()
    d.eps_m = 0 if eps_m_t is None else eps_m_t.data_ptr()
    d.seed, d.ctr = noise.seed, ctr
    d.rows_per_tile = getattr(alg, 'rows_per_tile', 0)
    engine = getattr(alg, 'rollout_engine', 0)
    if engine == 0:
        engine = 1 if (noise.parity and eps_layout == 0) or H > 128 else 2
    d.engine, d.eps_layout = engine, (eps_layout if noise.parity else 0)
    d.step_events = timer.events if timer is not None else None
    if timer is not None:
        timer.pairs = 1 if engine == 2 else H   # engine 2: one pair around the fused kernel
    _lib.check(L.drpo_rollout(ctypes.byref(d), _lib.stream()), 'rollout')
    vb._device_advanced()
    view = _RolloutResult(vb, start_ptr, count)
    view.tape_counts = ns
    return view


def rollout_host_env(alg, policy, initial_states, noise):
    """SMBPO.rollout (src/smbpo.py:229-249) for an env WITHOUT device constraint
    functions (envs.device_env_params returned None): the policy sample and the
    elite-member sample run on the HIP kernels, and the env's own numpy
    check_done / check_violation / get_constraint_values are called on the host each
    step -- the reference's round trip (src/smbpo.py:63-65), kept only for such envs."""
    from .buffers import ConstraintSafetySampleBuffer
    from .torch_util import torchify
    dev = alg.device
    B, H = alg.rollout_batch_size, alg.horizon
    S, A, C = alg.state_dim, alg.action_dim, alg.con_dim
    model, env = alg.model_ensemble, alg.real_env
    if initial_states is None:
        real = alg.replay_buffer.get('states', device=dev)
        idx = noise.np_choice(len(real), B)
        if idx is None:
            L = _lib.lib()
            idx_t = torch.empty(B, dtype=torch.int64, device=dev)
            _lib.check(L.drpo_sample_without_replacement(_lib.ptr(idx_t), B, len(real), noise.seed, noise.next(),
                                                         _lib.stream()), 'sample_without_replacement')
        else:
            idx_t = _dev(idx, dev, torch.int64)
        states = real.index_select(0, idx_t)
    else:
        states = initial_states.to(dev).float()
        B = len(states)
    buf = ConstraintSafetySampleBuffer(S, A, B * H, con_dim=C, device=dev)
    for t in range(H):
        actions = policy.act(states, eval=False, noise=noise)
        next_states, rewards = model.sample(states, actions, noise=noise)
        s2 = next_states.cpu().numpy()
        dones = torchify(env.check_done(s2), to_device=False).to(dev)
        viols = torchify(env.check_violation(s2), to_device=False).to(dev)
        h = torchify(env.get_constraint_values(s2), to_device=False).to(dev)
        buf.extend(states=states, actions=actions, next_states=next_states, rewards=rewards,
                   dones=dones.reshape(-1), violations=viols.reshape(-1), constraint_values=h.reshape(len(s2), *(
                       [] if C == 1 else [C])))
        continues = ~dones.reshape(-1).bool()
        if int(continues.sum()) == 0:
            break
        states = next_states[continues]
    alg.virt_buffer.extend(**buf.get(as_dict=True, device=dev))
    return buf


class _RolloutResult:
    def __init__(self, vb, start_ptr, count):
        self.vb, self._start, self._count = vb, start_ptr, count
        self.tape_counts = None

    def __len__(self):
        return int(self._count.item())

    def get(self, *names, as_dict=False, device=None):
        vb = self.vb
        names = names or vb.COMPONENT_NAMES
        n = len(self)
        end = vb.pointer
        start = end - n
        idx = (torch.arange(n, device=vb.device) + start) % vb.capacity
        out = [vb._bufs[k][idx] for k in names]
        if device is not None:
            out = [o.to(device) for o in out]
        if as_dict:
            return dict(zip(names, out))
        return out if len(out) > 1 else out[0]


# ---------------------------------------------------------------------------
# constraints / normalizer
# ---------------------------------------------------------------------------
def env_constraints(env_params, states):
    """Batched (done, violation, constraint_value) on the device; C==1 squeezed like torchify(np.squeeze(...))."""
    L = _lib.lib()
    _lib.require_device(states)
    states = states.contiguous().float()
    n, S = states.shape
    C = env_params['con_dim']
    done = torch.empty(n, dtype=torch.bool, device=states.device)
    viol = torch.empty(n, dtype=torch.bool, device=states.device)
    h = torch.empty(n, C, dtype=torch.float32, device=states.device)
    _lib.check(L.drpo_env_constraints(env_params['env_id'], env_params['tracking_surr_start'],
                                      env_params['tracking_n_surr'], env_params['thr0'],
                                      env_params['thr1'], _lib.ptr(states), n, S, _lib.ptr(done),
                                      _lib.ptr(viol), _lib.ptr(h), _lib.stream()), 'env_constraints')
    return done, viol, (h[:, 0] if C == 1 else h)


def normalizer_fit(X, mean, std):
    L = _lib.lib()
    _lib.require_device(X, mean, std)
    X = X.contiguous()
    N, S = X.shape
    ws = torch.empty(max(8, L.drpo_normalizer_workspace_size(N, S)), dtype=torch.uint8, device=X.device)
    _lib.check(L.drpo_normalizer_fit(_lib.ptr(X), N, S, _lib.ptr(mean), _lib.ptr(std), _lib.ptr(ws), _lib.stream()),
               'normalizer_fit')


def normalize(x, mean, std, eps):
    L = _lib.lib()
    _lib.require_device(x)
    x = x.contiguous()
    y = torch.empty_like(x)
    S = x.shape[-1]
    _lib.check(L.drpo_normalize(_lib.ptr(x), _lib.ptr(mean), _lib.ptr(std), float(eps), _lib.ptr(y),
                                x.numel() // S, S, _lib.stream()), 'normalize')
    return y


# ---------------------------------------------------------------------------
# stand-alone network forwards (policy act/distr, critics, multiplier): one fused
# MLP launch + one head launch each. Used outside the fused SAC step (real-env
# acting, evaluation, diagnostics) -- src/policy.py:76-100, src/ssac.py:17-111.
# ---------------------------------------------------------------------------
_default_noise = None


def default_noise():
    global _default_noise
    if _default_noise is None:
        from .rng import DeviceNoise
        _default_noise = DeviceNoise(torch.initial_seed() ^ 0xAC7)
    return _default_noise


def _mlp(nets, srcs, rows, trunk=False, norm=None, nbatch=1, sstride=None):
    from .sac_step import fill_fwd
    L = _lib.lib()
    d = fill_fwd(nets, srcs, rows, trunk=trunk, norm=norm, nbatch=nbatch, sstride=sstride)
    _lib.check(L.drpo_mlp_forward(ctypes.byref(d), _lib.stream()), 'mlp_forward')


def _net(group, prefix, spec, out_rows=None):
    from .sac_step import Net, spec_layers
    group.ensure_packed()
    net = Net(spec_layers(group, prefix, spec))
    if out_rows is not None:
        net.sy[-1] = torch.empty(out_rows, net.dout, device=group.data.device)
    return net


def _flat2(x, dim):
    x = x.contiguous().float()
    return x.reshape(-1, dim), x.shape[:-1]


def policy_raw(policy, states):
    _lib.require_device(policy.group.data, states)
    s, lead = _flat2(states, policy.state_dim)
    net = _net(policy.group, 'net.', policy.spec, len(s))
    _mlp([net], [(s, policy.state_dim)], len(s))
    return net.sy[-1], lead


def policy_act(policy, states, eval, noise=None):
    """TorchPolicy.act (src/policy.py:76-79): eval -> tanh(mu), else distr.sample()."""
    L = _lib.lib()
    raw, lead = policy_raw(policy, states)
    n, A = raw.shape[0], policy.action_dim
    a = torch.empty(n, A, device=raw.device)
    if eval:
        _lib.check(L.drpo_policy_head(_lib.ptr(raw), n, A, 2, None, 0, 0, 0, None, None, None, None, _lib.ptr(a),
                                      _lib.stream()), 'policy_head')
    else:
        noise = default_noise() if noise is None else noise
        eps = noise.normal((n, A))
        eps_t = None if eps is None else _dev(eps, raw.device)
        _lib.check(L.drpo_policy_head(_lib.ptr(raw), n, A, 0, _lib.ptr(eps_t), noise.seed, noise.next(), 9,
                                      _lib.ptr(a), None, None, None, None, _lib.stream()), 'policy_head')
    return a.reshape(*lead, A)


def policy_params(policy, states):
    """(loc, scale) of the squashed Gaussian (src/policy.py:88-97)."""
    L = _lib.lib()
    raw, lead = policy_raw(policy, states)
    n, A = raw.shape[0], policy.action_dim
    mu, sd = torch.empty(n, A, device=raw.device), torch.empty(n, A, device=raw.device)
    _lib.check(L.drpo_policy_head(_lib.ptr(raw), n, A, 3, None, 0, 0, 0, None, None, _lib.ptr(mu), _lib.ptr(sd),
                                  None, _lib.stream()), 'policy_head')
    return mu.reshape(*lead, A), sd.reshape(*lead, A)


def critic_all(critic, state, action, which=None):
    """CriticEnsemble.all (src/ssac.py:30-32): every Q net in one launch (grid.y = net);
    ``which`` restricts to a subset (random_choice, :38-40)."""
    _lib.require_device(critic.group.data, state, action)
    s, lead = _flat2(state, state.shape[-1])
    a, _ = _flat2(action, action.shape[-1])
    n = len(s)
    which = range(critic.n_critics) if which is None else which
    nets = [_net(critic.group, f'{critic.prefix}qs.{i}.', critic.spec, n) for i in which]
    for k in range(0, len(nets), 3):
        _mlp(nets[k:k + 3], [(s, s.shape[1]), (a, a.shape[1])], n)
    return [net.sy[-1].reshape(*lead) for net in nets]


def constraint_critic_forward(cc, state, action, uncertainty=False, sample=False, noise=None, repeat=1):
    """ConstraintCritic.forward (src/ssac.py:64-92): trunk + both heads in one launch,
    then the log-std clamp / quantile bound / clipped sample.

    repeat=K scores K action sets against the same states in ONE launch: ``action`` is
    [K*n, A] (set-major) and the states are read K times through a zero batch stride
    (the linear shield's candidates, src/sampling.py:430-437)."""
    assert not (uncertainty and sample), 'Uncertainty bound and sample cannot be True simultaneously.'
    L = _lib.lib()
    _lib.require_device(cc.group.data, state, action)
    s, lead = _flat2(state, state.shape[-1])
    a, _ = _flat2(action, action.shape[-1])
    if repeat > 1:
        assert len(a) == repeat * len(s), 'repeat: actions must be [repeat * n, A]'
        lead = (len(a),)
    n, C = len(a), cc.output_dim
    rows = len(s)
    trunk = _net(cc.group, cc.prefix + 'trunk.', cc.trunk_spec)
    mean = _net(cc.group, cc.prefix + 'mean_head.', cc.mean_spec, n)
    nets = [trunk, mean]
    if uncertainty or sample:
        nets.append(_net(cc.group, cc.prefix + 'log_std_head.', cc.logstd_spec, n))
    sstride = [0, rows * a.shape[1], 0] if repeat > 1 else None
    _mlp(nets, [(s, s.shape[1]), (a, a.shape[1])], rows, trunk=True, nbatch=repeat, sstride=sstride)
    shape = (*lead, C) if C > 1 else tuple(lead)
    mu = mean.sy[-1]
    if not (uncertainty or sample):
        return mu.reshape(shape)
    noise = default_noise() if noise is None else noise
    eps = noise.randn_like((n, C) if C > 1 else (n,), used=sample)
    eps_t = None if eps is None else _dev(eps, mu.device).reshape(n, C)
    q = torch.empty(n, C, device=mu.device)
    sd = torch.empty(n, C, device=mu.device) if sample else None
    _lib.check(L.drpo_cc_dist(_lib.ptr(mu), _lib.ptr(nets[2].sy[-1]), n * C, 1 if sample else 0, float(cc.std_ratio),
                              float(cc.log_std_min), float(cc.log_std_max), _lib.ptr(eps_t), noise.seed,
                              noise.next(), _lib.ptr(sd), _lib.ptr(q), _lib.stream()), 'cc_dist')
    if uncertainty:
        return q.reshape(shape)
    return mu.reshape(shape), sd.reshape(shape), q.reshape(shape)


# ---------------------------------------------------------------------------
# safety shields (src/smbpo.py:127-136, src/sampling.py:423-439)
# ---------------------------------------------------------------------------
SHIELD_NONE, SHIELD_THRESHOLD, SHIELD_LINEAR = 0, 1, 2


def shield_mix(a_perf, a_safe, K=11):
    """[K, n, A] candidates a_safe*(K-1-i)/(K-1) + a_perf*(1-(K-1-i)/(K-1))."""
    L = _lib.lib()
    _lib.require_device(a_perf, a_safe)
    a_perf, a_safe = a_perf.contiguous().float(), a_safe.contiguous().float()
    n, A = a_perf.shape
    mixes = torch.empty(K, n, A, device=a_perf.device)
    _lib.check(L.drpo_shield_mix(_lib.ptr(a_perf), _lib.ptr(a_safe), n, A, K, _lib.ptr(mixes), _lib.stream()),
               'shield_mix')
    return mixes


def shield_select(q, mode, threshold, a_perf, a_safe, mixes=None):
    """Per-row shield decision on the device; q [n(,C)] (mode 1) or [K*n(,C)] (mode 2)."""
    L = _lib.lib()
    _lib.require_device(q, a_perf, a_safe)
    a_perf, a_safe = a_perf.contiguous().float(), a_safe.contiguous().float()
    n, A = a_perf.shape
    K = 1 if mixes is None else mixes.shape[0]
    q = q.contiguous().float()
    C = q.numel() // (K * n) if mode == SHIELD_LINEAR else q.numel() // max(n, 1)
    out = torch.empty_like(a_perf)
    _lib.check(L.drpo_shield_select(_lib.ptr(q), K, n, max(C, 1), A, mode, float(threshold), _lib.ptr(a_perf),
                                    _lib.ptr(a_safe), _lib.ptr(mixes), _lib.ptr(out), _lib.stream()), 'shield_select')
    return out


def multiplier_forward(mult, state, Qc):
    """MLPMultiplier.forward (src/ssac.py:106-111)."""
    L = _lib.lib()
    _lib.require_device(mult.group.data, state, Qc)
    s, lead = _flat2(state, state.shape[-1])
    q = Qc.contiguous().float().reshape(-1, 1)
    n = len(s)
    net = _net(mult.group, 'lam.', mult.spec, n)
    _mlp([net], [(s, s.shape[1]), (q, 1)], n)
    lam = torch.empty(n, device=s.device)
    _lib.check(L.drpo_multiplier_out(n, _lib.ptr(net.sy[-1]), float(mult.upper_bound), _lib.ptr(lam), _lib.stream()),
               'multiplier_out')
    return lam.reshape(*lead)
