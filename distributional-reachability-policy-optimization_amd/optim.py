"""Optimizer state machines over flat parameter groups.

``Adam`` reproduces torch.optim.Adam (single-tensor path: coupled L2 weight decay,
lerp first moment, bias corrections formed in double on the host) and
``clip_grad_norm_`` semantics for the reference's separate clip groups; the
arithmetic runs in one HIP kernel per clip segment (csrc/optim.hip).
``CosineAnnealingLR`` reproduces torch's recursive (chainable) schedule, which is
host-side scalar logic in the reference too.
"""
import ctypes
import math

import torch

from . import _lib


class Adam:
    def __init__(self, group, lr, weight_decay=0.0, betas=(0.9, 0.999), eps=1e-8, tensor=None):
        """group: FlatGroup (or None with ``tensor`` = a flat fp32 tensor, e.g. log_alpha)."""
        self.group = group
        self.tensor = tensor
        self.betas, self.eps, self.weight_decay = betas, eps, weight_decay
        self.param_groups = [{'lr': lr, 'initial_lr': lr, 'weight_decay': weight_decay, 'betas': betas, 'eps': eps}]
        self.step_count = 0
        self.m = self.v = None

    @property
    def lr(self):
        return self.param_groups[0]['lr']

    def _data(self):
        return self.group.data if self.group is not None else self.tensor

    def _ensure_state(self):
        if self.m is None:
            d = self._data()
            self.m = torch.zeros_like(d)
            self.v = torch.zeros_like(d)

    def zero_grad(self):
        if self.group is not None:
            self.group.grad.zero_()

    def step_scalars(self):
        """Advance the step count; returns (lr/bc1, sqrt(bc2)) formed in double like torch."""
        self.step_count += 1
        b1, b2 = self.betas
        t = float(self.step_count)
        bc1 = 1 - b1 ** t
        bc2 = 1 - b2 ** t
        return self.lr / bc1, bc2 ** 0.5

    def apply(self, grad, start, end, scalars, clip=None, lr_scale=None):
        """Adam on elements [start, end) of the flat data with ``grad`` (same indexing);
        clip = (partial_sums_tensor, max_norm) or None."""
        self._ensure_state()
        d = self._data()
        _lib.require_device(d, grad)
        L = _lib.lib()
        n = end - start
        part, n_part, max_norm = (None, 0, 0.0) if clip is None else (clip[0], clip[0].numel(), clip[1])
        _lib.check(L.drpo_adam(_lib.ptr(d[start:end]), _lib.ptr(grad[start:end]), _lib.ptr(self.m[start:end]),
                               _lib.ptr(self.v[start:end]), n, scalars[0], scalars[1], self.betas[0],
                               self.betas[1], self.eps, self.weight_decay, _lib.ptr(part), n_part,
                               float(max_norm), _lib.ptr(lr_scale), _lib.stream()), 'adam')
        if self.group is not None:
            self.group.mark_dirty()

    def segment(self, start, end, scalars, clip=None, zero_grad=False, ema=None, pack_map=None, grad=None,
                grad_from_sum=None, grad_from_sum_kind=0, grad_scale=1.0):
        """drpo_optim_seg_t for elements [start, end) of this optimizer's tensor:
        clip = (partials, max_norm); ema = (target flat tensor, rate); pack_map = device
        drpo_pack_map_t of the group (refreshes its packed mirrors); grad_from_sum =
        (device sum, rows[, n]): gradient -c(p) * sum / rows of a scalar parameter (the sum
        of n device partials, added in order), with
        c = exp(p) (kind 0: the SAC temperature), sigmoid(p) (kind 1: the scalar
        multiplier's softplus) or 1 (kind 2: the log-alpha loss);
        grad_scale: multiplier of the gradient (and of its clip norm) -- 1/G after a
        data-parallel SUM all-reduce, so the mean needs no separate pass."""
        from ._abi import OptimSeg
        self._ensure_state()
        d = self._data()
        g = grad if grad is not None else (self.group.grad if self.group is not None else self.tensor.grad)
        sg = OptimSeg()
        sg.p, sg.g, sg.m, sg.v = d.data_ptr(), g.data_ptr(), self.m.data_ptr(), self.v.data_ptr()
        sg.start, sg.end, sg.adam = start, end, 1
        if clip is not None:
            sg.partial, sg.n_partial, sg.max_norm = clip[0].data_ptr(), clip[0].numel(), float(clip[1])
        sg.lr_over_bc1, sg.bc2_sqrt = scalars
        sg.beta1, sg.beta2 = self.betas
        sg.eps, sg.weight_decay = self.eps, self.weight_decay
        sg.zero_grad = int(zero_grad)
        if ema is not None:
            sg.ema_target, sg.ema_rate, sg.ema_keep = ema[0].data_ptr(), float(ema[1]), float(1.0 - float(ema[1]))
        sg.map = 0 if pack_map is None else pack_map.data_ptr()
        host = getattr(pack_map, 'host', None)
        sg.map_host = 0 if host is None else ctypes.addressof(host)
        if grad_from_sum is not None:
            sg.grad_from_sum, sg.grad_sum_rows = grad_from_sum[0].data_ptr(), int(grad_from_sum[1])
            sg.grad_from_sum_kind = int(grad_from_sum_kind)
            sg.grad_sum_n = int(grad_from_sum[2]) if len(grad_from_sum) > 2 else 1
        sg.grad_scale = float(grad_scale)
        return sg

    def step(self):
        """Plain step over the whole group (no clipping), for external training loops."""
        sc = self.step_scalars()
        d = self._data()
        g = self.group.grad if self.group is not None else self.tensor.grad
        self.apply(g, 0, d.numel(), sc)

    def state_dict(self):
        return {'step': self.step_count, 'm': self.m, 'v': self.v, 'param_groups': self.param_groups}

    def load_state_dict(self, sd):
        self.step_count = sd['step']
        self.m, self.v = sd['m'], sd['v']
        self.param_groups = sd['param_groups']


class CosineAnnealingLR:
    """torch.optim.lr_scheduler.CosineAnnealingLR, recursive form (torch 2.10)."""

    def __init__(self, optimizer, T_max, eta_min=0.0):
        self.optimizer, self.T_max, self.eta_min = optimizer, T_max, eta_min
        self.base_lr = optimizer.param_groups[0]['initial_lr']
        self.last_epoch = 0

    def step(self):
        self.last_epoch += 1
        e, T, eta = self.last_epoch, self.T_max, self.eta_min
        g = self.optimizer.param_groups[0]
        if (e - 1 - T) % (2 * T) == 0:
            g['lr'] = g['lr'] + (self.base_lr - eta) * (1 - math.cos(math.pi / T)) / 2
        else:
            g['lr'] = (1 + math.cos(math.pi * e / T)) / (1 + math.cos(math.pi * (e - 1) / T)) * (g['lr'] - eta) + eta

    def get_last_lr(self):
        return [self.optimizer.param_groups[0]['lr']]

    def state_dict(self):
        return {'last_epoch': self.last_epoch, 'base_lr': self.base_lr}

    def load_state_dict(self, sd):
        self.last_epoch, self.base_lr = sd['last_epoch'], sd['base_lr']


def grad_sumsq(grad_slice, workspace=None):
    """First pass of clip_grad_norm_: per-block partial sums of squares (device)."""
    L = _lib.lib()
    nb = L.drpo_grad_sumsq_blocks(grad_slice.numel())
    part = workspace[:nb] if workspace is not None else torch.empty(nb, device=grad_slice.device)
    _lib.check(L.drpo_grad_sumsq(_lib.ptr(grad_slice), grad_slice.numel(), _lib.ptr(part), _lib.stream()), 'sumsq')
    return part


def ema_(target, source, rate):
    L = _lib.lib()
    _lib.require_device(target, source)
    _lib.check(L.drpo_ema(_lib.ptr(target), _lib.ptr(source), target.numel(), float(rate), _lib.stream()), 'ema')


def ema_segment(p, start, end, target, rate, pack_map=None):
    """EMA-only segment (parameters not stepped by Adam, e.g. the vanilla log-std head)."""
    from ._abi import OptimSeg
    sg = OptimSeg()
    sg.p, sg.start, sg.end, sg.adam = p.data_ptr(), start, end, 0
    sg.ema_target, sg.ema_rate, sg.ema_keep = target.data_ptr(), float(rate), float(1.0 - float(rate))
    sg.map = 0 if pack_map is None else pack_map.data_ptr()
    host = getattr(pack_map, 'host', None)
    sg.map_host = 0 if host is None else ctypes.addressof(host)
    sg.grad_scale = 1.0
    return sg


OPT_MAXSEG = 8   # segments per drpo_optim_step launch (csrc/optim.hip)


def fused_step(segs):
    """drpo_optim_step over the given segments: one launch per 8 segments."""
    from ._abi import OptimSeg
    L = _lib.lib()
    for k in range(0, len(segs), OPT_MAXSEG):
        chunk = segs[k:k + OPT_MAXSEG]
        arr = (OptimSeg * len(chunk))(*chunk)
        _lib.check(L.drpo_optim_step(arr, len(chunk), _lib.stream()), 'optim_step')


def grad_sumsq_multi(slices, outs):
    """Partial sums of squares of several gradient slices in one launch."""
    import ctypes
    L = _lib.lib()
    n = len(slices)
    g = (ctypes.c_void_p * n)(*[t.data_ptr() for t in slices])
    cnt = (ctypes.c_int64 * n)(*[t.numel() for t in slices])
    o = (ctypes.c_void_p * n)(*[t.data_ptr() for t in outs])
    _lib.check(L.drpo_grad_sumsq_multi(g, cnt, o, n, _lib.stream()), 'grad_sumsq_multi')
