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


def rollout(alg, policy, initial_states, noise, timer=None):
    L = _lib.lib()
    dev = alg.device
    B, H = alg.rollout_batch_size, alg.horizon
    S, A, C = alg.state_dim, alg.action_dim, alg.con_dim
    model = alg.model_ensemble
    rb, vb = alg.replay_buffer._module, alg.virt_buffer._module
    assert B * H <= vb.capacity, 'We do not support extending by more than buffer capacity'
    _lib.require_device(policy.group.data, model.group.data, vb._states)

    # initial states: chronological replay indices (np.random.choice without replacement)
    if initial_states is not None:
        src, src_ptr, src_cap = initial_states.contiguous().float(), len(initial_states), len(initial_states)
        init_idx = torch.arange(B, device=dev, dtype=torch.int64)
    else:
        src, src_ptr, src_cap = rb._states, rb.pointer, rb.capacity
        n_real = min(src_ptr, src_cap)
        idx = noise.np_choice(n_real, B)
        init_idx = None if idx is None else _dev(idx, dev, torch.int64)

    S1 = S + 1
    if noise.parity:
        ks, ns, eps_a, eps_m = _tape_rollout_noise(noise, H, B, A, S1)
        members = [model._elite_inds[k] for k in ks] + [0] * (H - len(ks))
        eps_a_t, eps_m_t = _dev(eps_a, dev), _dev(eps_m, dev)
    else:
        ns = None
        members = [model._elite_inds[noise.choice(len(model._elite_inds))] for _ in range(H)]
        eps_a_t = eps_m_t = None
    ctr = noise.next()

    ws = alg._workspace('rollout', L.drpo_rollout_workspace_size(B, S, H))
    start_ptr = vb.pointer if vb._host_ptr is not None else None
    actor = policy.layers()
    trunk, diff, logv = model.views()
    ep = alg.env_params
    members_arr = (ctypes.c_int * H)(*members)
    d = RolloutDesc()
    d.S, d.A, d.C, d.Ha, d.Hm, d.B, d.H = S, A, C, policy.spec.dims[1], model.hidden_dim, B, H
    d.env_id, d.tracking_surr_start, d.tracking_n_surr = ep['env_id'], ep['tracking_surr_start'], ep['tracking_n_surr']
    d.quad_x_threshold, d.quad_z_threshold = ep['quad_x_threshold'], ep['quad_z_threshold']
    (d.aW1, d.ab1), (d.aW2, d.ab2), (d.aW3, d.ab3) = [(W.data_ptr(), b.data_ptr()) for W, b in actor]
    (d.mW1, d.mb1), (d.mW2, d.mb2) = [(W.data_ptr(), b.data_ptr()) for W, b in trunk]
    (d.dW1, d.db1), (d.dW2, d.db2) = [(W.data_ptr(), b.data_ptr()) for W, b in diff]
    (d.lW1, d.lb1), (d.lW2, d.lb2) = [(W.data_ptr(), b.data_ptr()) for W, b in logv]
    norm = model.state_normalizer
    d.norm_mean, d.norm_std = norm.mean.data_ptr(), norm.std.data_ptr()
    d.min_lv, d.max_lv = model.min_log_var.data_ptr(), model.max_log_var.data_ptr()
    d.members = members_arr
    d.replay_states, d.replay_ptr, d.replay_cap = src.data_ptr(), src_ptr, src_cap
    d.init_idx = 0 if init_idx is None else init_idx.data_ptr()
    d.eps_a = 0 if eps_a_t is None else eps_a_t.data_ptr()
    d.eps_m = 0 if eps_m_t is None else eps_m_t.data_ptr()
    d.seed, d.ctr = noise.seed, ctr
    d.vs, d.va, d.vs2, d.vr = vb._states.data_ptr(), vb._actions.data_ptr(), vb._next_states.data_ptr(), \
        vb._rewards.data_ptr()
    d.vh, d.vd, d.vv = vb._constraint_values.data_ptr(), vb._dones.data_ptr(), vb._violations.data_ptr()
    d.vptr, d.vcap = vb._pointer.data_ptr(), vb.capacity
    d.workspace = ws.data_ptr()
    d.rows_per_tile = getattr(alg, 'rows_per_tile', 0)
    d.step_events = timer.events if timer is not None else None
    _lib.check(L.drpo_rollout(ctypes.byref(d), _lib.stream()), 'rollout')
    vb._device_advanced()
    off = L.drpo_rollout_count_offset(B, S, H)
    count = ws[off:off + 8].view(torch.int64)[0]
    view = _RolloutResult(vb, start_ptr, count)
    view.tape_counts = ns
    return view


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
                                      env_params['tracking_n_surr'], env_params['quad_x_threshold'],
                                      env_params['quad_z_threshold'], _lib.ptr(states), n, S, _lib.ptr(done),
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
