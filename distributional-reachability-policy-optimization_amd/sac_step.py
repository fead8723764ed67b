"""SAC engine: the safe-SAC update (src/ssac.py:437-578, src/smbpo.py:251-279) as a
fixed sequence of HIP launches over engine-owned HBM workspaces.

Per update_solver call (DRPO flags, actor on, multiplier on) the device runs:
  sample_batch -> [critic] ONE multi-job forward ('c.f': the target critics and the
  target certificate chained behind the policies on s' in the same workgroups, the
  certificate on (s, a), the twin critics paired), ONE backward-data launch with the
  critic / certificate losses formed in-kernel ('c.b1'), ONE grouped weight-gradient
  launch (+ clip partials), ONE fused clip + Adam + EMA launch -> [actor] 'a.f1'
  (actor + safe actor paired, rsample heads), 'a.f2' (critics at (s, a), (s, a_safe),
  the certificate at tanh(mu_safe)), 'a.mult', 'a.b' (backward with the actor losses
  formed in-kernel), 'a.bpi' (both squashed-Gaussian backwards), ONE weight-gradient
  launch, ONE optimizer launch (+ alpha) -> [multiplier] 'm.f1', 'm.f2', 'm.mult',
  multiplier_head, backward, weight-gradient, optimizer.
All launch descriptors point at static workspaces, so they are built once per
batch size and the whole sequence is graph-capturable. Noise: Philox in the
kernels (production) or the reference's recorded draws (parity TapeNoise), which
are consumed here in the reference's call order.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._abi import (ActorHead, BufferView, CriticHead, MlpBwd, MlpFwd, SumDesc, WgradItem)
from .optim import ema_segment, fused_step, grad_sumsq_multi

ACT_ID = {None: 0, 'identity': 0, 'relu': 1, 'swish': 2, 'tanh': 3}

# Philox call-site ids (production noise)
SITE_PI_NEXT, SITE_SAFE_NEXT, SITE_PI_RS, SITE_SAFE_RS, SITE_PI_MULT = 1, 2, 5, 6, 8


def spec_layers(group, prefix, spec, buf=None):
    """[(P, b, din, dout, act, PT)] for an MLPSpec stored under prefix in a flat group:
    P / PT are the layer's packed forward / transposed weight mirrors (group.pview),
    b the bias view (of ``buf`` if given, else the group data)."""
    out = []
    n = spec.n_layers
    for i in range(n):
        act = spec.act if i < n - 1 else spec.out_act
        key = f'{prefix}{2 * i}.weight'
        b = group.view(f'{prefix}{2 * i}.bias', buf)
        PT = group.pview(key, True)
        out.append((group.pview(key)[0], b, spec.dims[i], spec.dims[i + 1], ACT_ID[act],
                    None if PT is None else PT[0]))
    return out


class Net:
    """One MLP as seen by the kernels: layer tuples + (optional) per-layer save buffers."""

    def __init__(self, layers, grad_layers=None):
        self.layers = layers              # [(P, b, din, dout, act, PT)]
        self.grad_layers = grad_layers    # [(gW, gb)] or None
        self.sy = [None] * len(layers)
        self.sz = [None] * len(layers)
        self.dz = [None] * len(layers)
        self.dz2 = [None] * len(layers)   # split-heads trunk: the second head's dZ share

    @property
    def dout(self):
        return self.layers[-1][3]

    @property
    def din(self):
        return self.layers[0][2]


def _p(t):
    return 0 if t is None else t.data_ptr()


def noise_tag(eps):
    """descriptor-cache suffix: recorded draws (parity) vs Philox (production)"""
    return '.p' if eps is not None else '.d'


def fill_net(dst, net, wstride=None):
    """drpo_mlp_net_t of a Net (layers, save buffers, per-member strides)."""
    dst.nl = len(net.layers)
    for l, (W, b, din, dout, act, WT) in enumerate(net.layers):
        L = dst.L[l]
        L.W, L.b, L.din, L.dout, L.act = W.data_ptr(), b.data_ptr(), din, dout, act
        L.sy, L.sz = _p(net.sy[l]), _p(net.sz[l])
        L.wstride, L.bstride = (0, 0) if wstride is None else wstride[l]


def fill_fwd(nets, srcs, rows, trunk=False, save_x=None, norm=None, nbatch=1, wstride=None, sstride=None,
             split_heads=False, pair=False):
    """pair: the two nets run by one workgroup (multi-job launches; drpo_mlp_fwd_t.pair)."""
    d = MlpFwd()
    for k, (t, cols) in enumerate(srcs):
        d.src[k] = _p(t)
        d.cols[k] = cols
        d.ld[k] = t.shape[-1] if t is not None and t.dim() > 1 else 1
        d.sstride[k] = 0 if sstride is None else sstride[k]
    d.nmean, d.nstd = (norm[0].data_ptr(), norm[1].data_ptr()) if norm is not None else (0, 0)
    d.save_x = _p(save_x)
    for j, net in enumerate(nets):
        fill_net(d.net[j], net, None if wstride is None else wstride[j])
    d.nnets, d.trunk, d.rows, d.nbatch = len(nets), int(trunk), rows, nbatch
    d.split_heads = int(split_heads)
    d.pair = int(pair)
    return d


def pairable(a, b):
    """Two nets one pair job can run (csrc/mlp.hip pair_ok): 3-layer ReLU nets of one shape
    [K <= 16 or 49..64 -> 256 -> 256 -> <= 16] (the reference's default widths)."""
    la, lb = a.layers, b.layers
    if len(la) != 3 or len(lb) != 3:
        return False
    if any(x[2:5] != y[2:5] for x, y in zip(la, lb)):
        return False
    (_, _, k0, n0, a0, _), (_, _, k1, n1, a1, _), (_, _, _, n2, a2, _) = la
    return ((k0 + 15) // 16 in (1, 4) and n0 == 256 and k1 == 256 and n1 == 256 and n2 <= 16 and
            a0 == ACT_ID['relu'] and a1 == ACT_ID['relu'] and a2 == 0)


def with_pre(d, policy, mode, A, eps, site, logp=None):
    """Chain (drpo_mlp_fwd_t.pre): the policy runs first in the same workgroup on the
    src[0] columns; its sampled action (mode 1 sample / 2 rsample) is the job's src[1]
    block, straight from LDS."""
    fill_net(d.pre, policy)
    h = d.pre_head
    h.mode, h.A, h.eps, h.site, h.logp = mode, A, _p(eps), site, _p(logp)
    return d


def with_post(d, net, post_x=None):
    """Post chain (drpo_mlp_fwd_t.post): `net` (the MLPMultiplier) runs after the job's
    constraint bound (ccb_out), in the same workgroup, on [src[0] columns, bound]; its
    layers save as any net's, post_x saves the assembled input (the multiplier update's
    weight-gradient Y)."""
    fill_net(d.post, net)
    d.post_x = _p(post_x)
    return d


# drpo_mlp_bwd_t.upstream (include/drpo_hip.h DRPO_UPSTREAM_*)
UPSTREAM_GOUT, UPSTREAM_CRITIC, UPSTREAM_CERT, UPSTREAM_ENS = 0, 1, 2, 3
UPSTREAM_ACTOR_CC, UPSTREAM_SAFE_CC, UPSTREAM_NEG_MEAN, UPSTREAM_SQUASH, UPSTREAM_SQUASH_SAFE = 4, 5, 6, 7, 8


def fill_bwd(nets, gouts, rows, trunk=False, dx=None, nbatch=1, wstride=None, split_heads=False, upstream=0):
    """nets[0] trunk when trunk=True (gouts[0] ignored); dx: {net_index: (tensor, col0, cols, accumulate)};
    split_heads: one workgroup per head, the second head's trunk dZ share into nets[0].dz2;
    upstream: output gradients from the gout arrays, or formed in-kernel from the
    launch's critic head (UPSTREAM_CRITIC / UPSTREAM_CERT)."""
    d = MlpBwd()
    d.upstream = upstream
    for j, net in enumerate(nets):
        d.net[j].nl = len(net.layers)
        for l, (W, b, din, dout, act, WT) in enumerate(net.layers):
            L = d.net[j].L[l]
            assert WT is not None, 'backward needs the transposed weight mirror (trained group)'
            L.W, L.din, L.dout, L.act = WT.data_ptr(), din, dout, act
            L.sy, L.sz, L.dz = _p(net.sy[l]), _p(net.sz[l]), _p(net.dz[l])
            L.dz2 = _p(net.dz2[l]) if getattr(net, 'dz2', None) else 0
            L.wstride = 0 if wstride is None else wstride[j][l][0]
        d.net[j].gout = _p(gouts[j])
        if dx and j in dx:
            t, c0, nc, accum = dx[j]
            d.net[j].dx, d.net[j].dx_col0, d.net[j].dx_cols, d.net[j].dx_accumulate = t.data_ptr(), c0, nc, int(accum)
    d.nnets, d.trunk, d.rows, d.nbatch = len(nets), int(trunk), rows, nbatch
    d.split_heads = int(split_heads)
    return d


HEAD_SAMPLE, HEAD_RSAMPLE, HEAD_MEAN = 1, 2, 3


def with_head(d, mode, A, eps, site, a=None, logp=None, u=None, e=None, amean=None, second=False):
    """Attach a fused squashed-Gaussian head (drpo_policy_head_t) to a forward descriptor
    (second: the head of a pair job's net 1, drpo_mlp_fwd_t.head2)."""
    h = d.head2 if second else d.head
    h.mode, h.A, h.eps, h.site = mode, A, _p(eps), site
    h.a, h.logp, h.u, h.e, h.amean = _p(a), _p(logp), _p(u), _p(e), _p(amean)
    return d


def wgrad_items(entries, rows, sq=None):
    """entries: [(net, inputs_per_layer[, segment])] -> (ctypes array of WgradItem, count,
    {segment: partial slots used}). With sq = {segment: device tensor}, every item of a
    segment writes the sums of squares of its finished gradient tiles into consecutive
    slots of that segment's tensor (the clip partials of drpo_optim_step)."""
    L = _lib.lib()
    items, used = [], {}
    units = [(ent[0], ent[1], ent[2] if len(ent) > 2 else None, l) for ent in entries for l in range(len(ent[0].layers))]
    for net, ins, seg, l in units:
        W, b, din, dout, act, WT = net.layers[l]
        gW, gb = net.grad_layers[l]
        it = WgradItem()
        it.dz, it.y, it.gW, it.gb = net.dz[l].data_ptr(), ins[l].data_ptr(), gW.data_ptr(), gb.data_ptr()
        it.dout, it.din, it.rows, it.nbatch = dout, din, rows, 1
        if sq is not None and seg is not None:
            it.sq, it.sq_off = sq[seg].data_ptr(), used.get(seg, 0)
            used[seg] = it.sq_off + L.drpo_mlp_wgrad_tiles(ctypes.byref(it))
            assert used[seg] <= sq[seg].numel(), 'clip partial buffer too small'
        items.append(it)
    arr = (WgradItem * len(items))(*items)
    return arr, len(items), used


def wgrad_workspace(cache, key, arr, n, dev):
    """Zero-initialised workspace of one drpo_mlp_wgrad call site (the launches keep it
    zeroed), cached by key and grown when the plan needs more."""
    need = int(_lib.lib().drpo_mlp_wgrad_workspace_size(arr, n))
    t = cache.get(key)
    if t is None or t.numel() < need:
        t = torch.zeros(max(need, 256), dtype=torch.uint8, device=dev)
        cache[key] = t
    return t


def fwd_flops(d):
    """Algorithmic FLOPs of one drpo_mlp_forward launch (2 * rows * sum din*dout), the
    chained policy and the post-chain multiplier of a multi-job launch included."""
    macs = 0
    for n in [d.net[j] for j in range(d.nnets)] + [d.pre, d.post]:
        for l in range(n.nl):
            macs += n.L[l].din * n.L[l].dout
    return 2 * d.rows * d.nbatch * macs


def bwd_flops(d):
    """Backward-data products (dY = dZ W) of one drpo_mlp_backward launch; layer 0's
    product runs only for trunk-mode heads (it feeds the trunk) or when the input
    gradient is requested."""
    macs = 0
    for j in range(d.nnets):
        n = d.net[j]
        for l in range(n.nl):
            if l > 0 or n.dx or (d.trunk and j > 0):
                macs += n.L[l].din * n.L[l].dout
    return 2 * d.rows * d.nbatch * macs


def wgrad_flops(arr, n):
    # (arr, n[, used]) descriptors
    return sum(2 * arr[i].rows * arr[i].nbatch * arr[i].dout * (arr[i].din + 1) for i in range(n))


class LaunchProfiler:
    """HIP events around every MLP launch of the engine (stream-ordered on the launch
    stream), with each launch's algorithmic FLOPs; summarise() after a synchronize."""

    def __init__(self):
        self.recs = []

    def begin(self, kind, key, flops):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        return (kind, key, flops, e0, e1)

    def end(self, rec):
        rec[4].record()
        self.recs.append(rec)

    def summarise(self):
        out = {}
        for kind, key, flops, e0, e1 in self.recs:
            ms = e0.elapsed_time(e1)
            for k in (kind, f'{kind}:{key}'):
                o = out.setdefault(k, {'launches': 0, 'ms': 0.0, 'flop': 0.0})
                o['launches'] += 1
                o['ms'] += ms
                o['flop'] += flops
        for o in out.values():
            o['avg_ms'] = o['ms'] / o['launches']
            o['tflops'] = o['flop'] / (o['ms'] * 1e-3) / 1e12 if o['ms'] > 0 else 0.0
        self.recs = []
        return out


class SACEngine:
    def __init__(self, solver):
        self.sol = solver
        self.profiler = None
        # C: the constraint critic's output width (con_dim, or 1 for the cost certificate);
        # Ch: the constraint values' width (the batch's h)
        self.S, self.A, self.C = solver.state_dim, solver.action_dim, solver.constraint_critic.output_dim
        self.Ch = solver.con_dim
        self.cost = solver.constrained_fcn == 'cost'
        self.dev = solver.actor.group.data.device
        from .distributed import GradReducer
        self.dp = GradReducer()
        from .envs import device_env_params
        self.env_params = device_env_params(solver.env) if solver.qc_under_uncertainty and \
            not solver.distributional_qc and not self.cost else None
        self.B = None
        self.ws = {}
        self.wg_ws = {}
        # The actor update's data-parallel exchange is ONE all-reduce:
        # the actor's and the safe actor's flat gradients and the alpha-loss sum are
        # adjacent slices of one arena (the critic and multiplier phases already exchange
        # one flat buffer each).
        # the alpha-loss sum travels as its per-16-row-tile partials (written, not
        # accumulated, by the squash backward; summed in order by the optimizer launch)
        self.actor_xchg = None
        self._actor_arena(solver.batch_size)
        self.loss_pool = None
        self.loss_pos = 0
        self._zeroed = set()   # groups whose grads the last fused step left zeroed
        self.noise = None
        # production dispatch: the MLPMultiplier forward as a post chain of the bound's job
        # (False: its own launch, the reference of
        # tests/test_gpu_configs.py::test_multiplier_post_chain_matches_separate_launch)
        self.post_mult = True

    # ------------------------------------------------------------------ buffers
    def buf(self, name, *shape, dtype=torch.float32):
        t = self.ws.get(name)
        if t is None or tuple(t.shape) != tuple(shape) or t.dtype != dtype:
            t = torch.zeros(*shape, dtype=dtype, device=self.dev)
            self.ws[name] = t
        return t

    def _loss_slots(self, n):
        if self.loss_pool is None or self.loss_pos + n > self.loss_pool.numel():
            self.loss_pool = torch.zeros(1 << 16, device=self.dev)
            self.loss_pos = 0
        s = self.loss_pool[self.loss_pos:self.loss_pos + n]
        self.loss_pos += n
        return s

    def _actor_arena(self, B):
        """(Re)build the actor exchange arena for batch B: actor grads | safe actor grads |
        one alpha-loss partial per 16-row tile. Sized once for the solver's batch size
        (and never below 4096 rows); a larger B re-homes the gradients, which re-points
        the Parameters' .grad views and drops every cached descriptor and net view (they
        hold raw pointers into the old arena)."""
        nt = (B + 15) // 16
        if self.actor_xchg is not None and self.alpha_sum.numel() >= nt:
            return
        sol = self.sol
        nt = max(nt, (max(sol.batch_size, 4096) + 15) // 16)
        if self.actor_xchg is not None:
            nt = max(nt, 2 * self.alpha_sum.numel())   # grow geometrically: rare rebuilds
        ga, gs = sol.actor.group, sol.actor_safe.group
        na, ns = ga.size, gs.size
        self.actor_xchg = torch.zeros(na + ns + nt, device=self.dev)
        ga.move_grad(self.actor_xchg[:na], sol.actor)
        gs.move_grad(self.actor_xchg[na:na + ns], sol.actor_safe)
        self.alpha_sum = self.actor_xchg[na + ns:]
        self.desc = {}
        self.nets_view = {}
        self.B = None          # forces _setup to rebuild the nets over the new gradient views

    def _setup(self, B):
        if self.B == B:
            return
        self._actor_arena(B)
        self.B = B
        self.ws = {}
        sol, S, A, C = self.sol, self.S, self.A, self.C
        cg, tg = sol.critic_group, sol.critic_target_group
        ag, sg, mg = sol.actor.group, sol.actor_safe.group, sol.multiplier_group
        cspec, ccs = sol.critic.spec, sol.constraint_critic
        buf = self.buf

        def mk(group, prefix, spec, grads=True, data=None):
            lay = spec_layers(group, prefix, spec, data)
            gl = None
            if grads:
                gl = [(g[0], g[1]) for g in ((group.view(f'{prefix}{2 * i}.weight', group.grad),
                                              group.view(f'{prefix}{2 * i}.bias', group.grad))
                                             for i in range(spec.n_layers))]
            return Net(lay, gl)

        self.nets = n = {}
        n['actor'] = mk(ag, 'net.', sol.actor.spec)
        n['safe'] = mk(sg, 'net.', sol.actor_safe.spec)
        n['q0'] = mk(cg, 'critic.qs.0.', cspec)
        n['q1'] = mk(cg, 'critic.qs.1.', cspec)
        n['q0t'] = mk(tg, 'critic.qs.0.', cspec, grads=False)
        n['q1t'] = mk(tg, 'critic.qs.1.', cspec, grads=False)
        for tag, grp, gr in (('', cg, True), ('t', tg, False)):
            n['cc_trunk' + tag] = mk(grp, 'constraint_critic.trunk.', ccs.trunk_spec, gr)
            n['cc_mean' + tag] = mk(grp, 'constraint_critic.mean_head.', ccs.mean_spec, gr)
            n['cc_ls' + tag] = mk(grp, 'constraint_critic.log_std_head.', ccs.logstd_spec, gr)
        if sol.mlp_multiplier:
            n['mult'] = mk(mg, 'lam.', sol.multiplier.spec)
        self.nets_view = {}
        # forward saves (post-activations) and dz for every trained net
        for key, net in n.items():
            if net.grad_layers is None:
                continue
            for l, (_, _, din, dout, act, _) in enumerate(net.layers):
                net.sy[l] = buf(f'{key}.sy{l}', B, dout)
                net.dz[l] = buf(f'{key}.dz{l}', B, dout)
        for key in ('q0t', 'q1t', 'cc_trunkt', 'cc_meant', 'cc_lst'):
            net = n[key]
            net.sy[-1] = buf(f'{key}.out', B, net.dout)
        # batch
        self.bs, self.ba, self.bs2 = buf('b.s', B, S), buf('b.a', B, A), buf('b.s2', B, S)
        self.br, self.bh = buf('b.r', B), buf('b.h', B, self.Ch)
        self.bd, self.bv = buf('b.d', B, dtype=torch.uint8), buf('b.v', B, dtype=torch.uint8)
        # noise buffers (parity mode)
        for k, shp in (('em', (B, S + 1)), ('e1', (B, A)), ('e2', (B, A)), ('e3', (B, C)), ('e5', (B, A)), ('e6', (B, A)),
                       ('e7', (B, A))):
            buf(k, *shp)
        buf('idx_r', B, dtype=torch.int64)
        buf('idx_v', B, dtype=torch.int64)
        self.desc = {}

    # ------------------------------------------------------------------ noise
    def _eps(self, name, arr):
        if arr is None:
            return None
        t = self.ws[name]
        t.view(-1)[:arr.size].copy_(torch.from_numpy(np.ascontiguousarray(arr, np.float32)).view(-1))
        return t

    # ------------------------------------------------------------------ helpers
    def _ensure_packed(self):
        """Refresh the packed weight mirrors of every group an update step reads."""
        sol = self.sol
        for g in (sol.actor.group, sol.actor_safe.group, sol.critic_group, sol.critic_target_group,
                  sol.multiplier_group):
            g.ensure_packed()

    def _run_fwd(self, key, builder):
        d = self.desc.get(key)
        if d is None:
            d = self.desc[key] = builder()
        ev = self.profiler.begin('mlp_fwd', key, fwd_flops(d)) if self.profiler else None
        _lib.check(_lib.lib().drpo_mlp_forward(ctypes.byref(d), _lib.stream()), key)
        if ev:
            self.profiler.end(ev)

    def _upload(self, structs):
        raw = bytes(structs)
        return torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.dev)

    def _run_multi(self, key, builder, ctr):
        """Independent forwards (+ fused policy heads) in one launch; descriptors are
        built once and kept in device memory."""
        d = self.desc.get(key)
        if d is None:
            jobs = builder()
            arr = (MlpFwd * len(jobs))(*jobs)
            d = self.desc[key] = (arr, self._upload(arr), len(jobs), sum(fwd_flops(j) for j in jobs))
        arr, dev, nj, fl = d
        ev = self.profiler.begin('mlp_fwd', key, fl) if self.profiler else None
        _lib.check(_lib.lib().drpo_mlp_forward_multi(arr, dev.data_ptr(), nj, self.noise.seed, ctr, _lib.stream()), key)
        if ev:
            self.profiler.end(ev)

    def _run_bwd_multi(self, key, builder, head=None, actor=None):
        d = self.desc.get(key)
        if d is None:
            jobs = builder()
            arr = (MlpBwd * len(jobs))(*jobs)
            d = self.desc[key] = (arr, self._upload(arr), len(jobs), sum(bwd_flops(j) for j in jobs))
        arr, dev, nj, fl = d
        ev = self.profiler.begin('mlp_bwd', key, fl) if self.profiler else None
        if actor is not None:
            _lib.check(_lib.lib().drpo_mlp_backward_multi_actor(arr, dev.data_ptr(), nj, ctypes.byref(actor),
                                                                _lib.stream()), key)
        elif head is None:
            _lib.check(_lib.lib().drpo_mlp_backward_multi(arr, dev.data_ptr(), nj, _lib.stream()), key)
        else:
            _lib.check(_lib.lib().drpo_mlp_backward_multi_head(arr, dev.data_ptr(), nj, ctypes.byref(head),
                                                               _lib.stream()), key)
        if ev:
            self.profiler.end(ev)

    def _run_bwd(self, key, builder):
        d = self.desc.get(key)
        if d is None:
            d = self.desc[key] = builder()
        ev = self.profiler.begin('mlp_bwd', key, bwd_flops(d)) if self.profiler else None
        _lib.check(_lib.lib().drpo_mlp_backward(ctypes.byref(d), _lib.stream()), key)
        if ev:
            self.profiler.end(ev)

    def _run_wgrad(self, key, builder, sums=None):
        """One grouped weight-gradient launch; returns the clip-partial slots per segment.
        sums: [(partials, out)] -- loss partials the launch's extra block adds up in order
        into the 0-d `out` (drpo_mlp_wgrad_sums)."""
        d = self.desc.get(key)
        if d is None:
            arr, n, used = builder()
            ws = wgrad_workspace(self.wg_ws, key, arr, n, self.dev)
            d = self.desc[key] = (arr, n, used, ws, (SumDesc * 4)())
        arr, n, used, ws, sd = d
        ev = self.profiler.begin('mlp_wgrad', key, wgrad_flops(arr, n)) if self.profiler else None
        if sums:
            for q, (part, out) in enumerate(sums):
                sd[q].part, sd[q].n, sd[q].out = part.data_ptr(), part.numel(), out.data_ptr()
            _lib.check(_lib.lib().drpo_mlp_wgrad_sums(arr, n, sd, len(sums), ws.data_ptr(), ws.numel(),
                                                      _lib.stream()), key)
        else:
            _lib.check(_lib.lib().drpo_mlp_wgrad(arr, n, ws.data_ptr(), ws.numel(), _lib.stream()), key)
        if ev:
            self.profiler.end(ev)
        return used

    def _clip_parts(self, fused, key, segs, grads):
        """Clip partial sums per segment: from the weight-gradient launch (fused, single
        process) or, after a data-parallel all-reduce, one sum-of-squares launch over
        the reduced gradient slices."""
        if fused is not None:
            return [self.buf(f'sq.{key}.{sg}', 4096)[:fused[sg]] for sg in segs]
        L = _lib.lib()
        parts = [self.buf(f'part.{key}.{sg}', 4096)[:L.drpo_grad_sumsq_blocks(g.numel())] for sg, g in zip(segs, grads)]
        grad_sumsq_multi(grads, parts)
        return parts

    def _sq(self, key, segs):
        """{segment: partial buffer} for a fused-clip weight-gradient launch, or None
        under data parallelism (the norm must be of the all-reduced gradient)."""
        if self.dp.active:
            return None
        return {sg: self.buf(f'sq.{key}.{sg}', 4096) for sg in segs}

    def _policy_head(self, raw, mode, eps, site, ctr, a=None, logp=None, u=None, e=None, amean=None):
        L = _lib.lib()
        seed = self.noise.seed
        _lib.check(L.drpo_policy_head(raw.data_ptr(), self.B, self.A, mode, _p(eps), seed, ctr, site, _p(a), _p(logp),
                                      _p(u), _p(e), _p(amean), _lib.stream()), 'policy_head')

    def _ccb_fused(self):
        """The multi-job forward can form the bound when the constraint critic's heads are
        pairable (256-wide trunk, two [256 -> H -> C <= 16] heads: the reference widths)."""
        t, h1, h2 = self._cc_nets()
        (_, _, _, tw, _, _), l1, l2 = t.layers[-1], h1.layers, h2.layers
        return (tw == 256 and len(l1) == 2 and len(l2) == 2 and l1[0][3] == l2[0][3] and l1[1][3] <= 16
                and l2[1][3] <= 16 and l1[0][4] == l2[0][4] and l1[1][4] == l2[1][4])

    def _ccb(self, d, out, dist):
        """The constraint critic's max-C upper bound (drpo_cc_head's arithmetic) formed
        by the multi-job forward from the paired heads' outputs (drpo_mlp_fwd_t.ccb_*);
        other head shapes keep the drpo_cc_head launch (_cc_bound_after)."""
        if not self._ccb_fused():
            return d
        cc = self.sol.constraint_critic
        d.ccb_out, d.ccb_dist = out.data_ptr(), int(dist)
        d.ccb_ratio, d.ccb_lmin, d.ccb_lmax = float(cc.std_ratio), float(cc.log_std_min), float(cc.log_std_max)
        return d

    def _post_mult(self):
        """The multiplier forward as a post chain of the bound's job (csrc/mlp.hip,
        drpo_mlp_fwd_t.post) when the shapes allow it (self.post_mult)."""
        return (self.post_mult and self._ccb_fused() and self.S + 1 <= 64 and
                self.nets['mult'].layers[0][2] == self.S + 1)

    def _cc_bound_after(self, name, out, dist):
        """drpo_cc_head over the saved head outputs of job `name` when _ccb could not fuse it."""
        if self._ccb_fused():
            return
        cc = self.sol.constraint_critic
        mu, ls = self.ws[f'{name}.mu'], self.ws[f'{name}.ls']
        _lib.check(_lib.lib().drpo_cc_head(mu.data_ptr(), ls.data_ptr(), self.B, self.C, int(dist), float(cc.std_ratio),
                                           float(cc.log_std_min), float(cc.log_std_max), out.data_ptr(), None,
                                           _lib.stream()), 'cc_head')

    def _clean_grads(self, group):
        """Gradients must be zero before the backward passes accumulate into them; the
        fused optimizer step leaves them zeroed, so this only clears after anything else."""
        if group.name not in self._zeroed:
            group.grad.zero_()
        self._zeroed.discard(group.name)

    def _grads_zeroed(self, group):
        self._zeroed.add(group.name)

    def _alive_span(self, group, prefixes):
        spans = [group.span(p) for p in prefixes]
        return min(s[0] for s in spans), max(s[1] for s in spans)

    def _cc_nets(self, tag=''):
        n = self.nets
        return [n['cc_trunk' + tag], n['cc_mean' + tag], n['cc_ls' + tag]]

    # ------------------------------------------------------------------ updates
    def update_critic(self, obs, action, next_obs, reward, done, violation, constraint_value, noise=None):
        """SSAC.update_critic (src/ssac.py:437-456). Returns (critic_loss, constraint_critic_loss) 0-d tensors."""
        B = obs.shape[0]
        self._setup(B)
        for dst, src in ((self.bs, obs), (self.ba, action), (self.bs2, next_obs), (self.br, reward)):
            dst.copy_(src.reshape(dst.shape))
        self.bd.copy_(done.reshape(B).to(torch.uint8))
        self.bv.copy_(violation.reshape(B).to(torch.uint8))
        self.bh.copy_(constraint_value.reshape(B, self.Ch))
        return self._critic_step(noise)

    def _critic_step(self, noise, early_actor=False):
        sol, n, B, S, A, C = self.sol, self.nets, self.B, self.S, self.A, self.C
        self._ensure_packed()
        self.noise = noise = noise or self.noise
        L = _lib.lib()
        dist = sol.distributional_qc and sol.qc_under_uncertainty
        robust = sol.qc_under_uncertainty and not sol.distributional_qc and not self.cost
        qshape = (B,) if C == 1 else (B, C)
        e1 = self._eps('e1', noise.normal((B, A)))
        if robust:
            # robust certificate target (src/ssac.py:387-400): s' drawn from one elite
            # member of the dynamics model, done flags from the env's constraint fns
            model = sol.model_ensemble
            member = model._elite_inds[noise.choice(len(model._elite_inds))]
            em = self._eps('em', noise.randn_like((B, S + 1)))
        e2 = self._eps('e2', noise.normal((B, A)))
        e3 = self._eps('e3', noise.randn_like(qshape)) if dist else None
        noise.randn_like(qshape, used=False)       # loss forward's unused draw (src/ssac.py:80)
        ctr = noise.next()
        ws = self.ws
        s2c, rk = self.bs2, ''
        if robust:
            s2c, rk = self.buf('c.s2m', B, S), '.r'
            model.engine.sample(self.bs, self.ba, member, noise, eps=em, tag='sac',
                                out={'s2': s2c, 'r': self.buf('c.r2m', B)})
            dm = self.buf('c.dm', B, dtype=torch.uint8)
            ep = self.env_params
            if ep is None:
                # env without device constraint fns: the reference's host round trip
                # (src/ssac.py:389, env.check_done on the model's s')
                done_h = np.asarray(sol.env.check_done(s2c.detach().cpu().numpy())).reshape(B)
                dm.copy_(torch.from_numpy(done_h.astype(np.uint8)))
            else:
                _lib.check(L.drpo_env_constraints(ep['env_id'], ep['tracking_surr_start'], ep['tracking_n_surr'],
                                                  ep['thr0'], ep['thr1'], s2c.data_ptr(), B, S,
                                                  dm.data_ptr(), self.buf('c.vm', B, dtype=torch.uint8).data_ptr(),
                                                  self.buf('c.hm', B, C).data_ptr(), _lib.stream()),
                           'env_constraints')
        xs = self.buf('c.x', B, S + A)
        lp2 = self.buf('c.lp2', B)
        # ONE launch (jobs longest chain first: workgroups dispatch in slot order, so the
        # short chains fill the tail): the constraint critic and the twin critics (one
        # workgroup for both twins) at (s, a) with their backward saves, and the targets with
        # their next-state policies chained in (drpo_mlp_fwd_t.pre): a'_safe ~ pi_safe(s')
        # (robust: the model's s') -> target certificate at (s', a'_safe); a' ~ pi(s') with
        # log pi -> target twins at (s', a') (src/ssac.py:284-294,304-400). The cost certificate
        # draws its next action from the actor instead (src/ssac.py:306-310).
        pq = pairable(n['q0'], n['q1'])
        tpol = n['actor' if self.cost else 'safe']
        # early_actor: the following actor update's first forward (actor / safe-actor
        # rsample, independent of the critic update) rides in this launch as its shortest
        # job, drawing its Philox noise at this launch's counter (device noise only)
        # Job order = workgroup dispatch order. Measured (profiles/r05/early_actor): without
        # the actor jobs, q pair, certificate, qt chain, cc_t chain (94.3 us; cc_t, qt, cc, q
        # 97.2; cc, q, cc_t, qt 100.4); with them, actor, certificate, q pair, cc_t, qt
        # (105.5 us; actor, q, cc, qt, cc_t 112.9; actor, chains, plain 111.4; chains, plain,
        # actor 119.5).

        def cf_jobs():
            chains = [with_pre(fill_fwd(self._cc_nets('t'), [(s2c, S), (None, A), (None, 0)], B, trunk=True),
                               Net(tpol.layers), HEAD_SAMPLE, A, e2, SITE_SAFE_NEXT),
                      with_pre(fill_fwd([n['q0t'], n['q1t']], [(self.bs2, S), (None, A), (None, 0)], B, pair=pq),
                               Net(n['actor'].layers), HEAD_SAMPLE, A, e1, SITE_PI_NEXT, logp=lp2)]
            plain = [fill_fwd(self._cc_nets(), [(self.bs, S), (self.ba, A), (None, 0)], B, trunk=True),
                     fill_fwd([n['q0'], n['q1']], [(self.bs, S), (self.ba, A), (None, 0)], B, save_x=xs, pair=pq)]
            if early_actor:   # actor, certificate, q pair, cc_t chain, qt chain
                return self._actor_f1_jobs(None, None) + plain + chains
            return plain[::-1] + chains[::-1]          # q pair, certificate, qt chain, cc_t chain
        self._run_multi('c.f' + rk + noise_tag(e1) + ('+a' if early_actor else ''), cf_jobs, ctr)
        loss = self._loss_slots(2)
        self._clean_grads(sol.critic_group)
        ch = self.desc.get('c.head')
        if ch is None:
            ch = self.desc['c.head'] = CriticHead()
            ch.B, ch.C = B, C
            ch.r, ch.h, ch.d = self.br.data_ptr(), self.bh.data_ptr(), self.bd.data_ptr()
            ch.q0t, ch.q1t, ch.logp2 = n['q0t'].sy[-1].data_ptr(), n['q1t'].sy[-1].data_ptr(), ws['c.lp2'].data_ptr()
            ch.mu_t, ch.ls_t = n['cc_meant'].sy[-1].data_ptr(), n['cc_lst'].sy[-1].data_ptr()
            ch.q0, ch.q1 = n['q0'].sy[-1].data_ptr(), n['q1'].sy[-1].data_ptr()
            ch.mu, ch.ls = n['cc_mean'].sy[-1].data_ptr(), n['cc_ls'].sy[-1].data_ptr()
            ch.dq0, ch.dq1 = self.buf('c.dq0', B).data_ptr(), self.buf('c.dq1', B).data_ptr()
            ch.dmu, ch.dls = self.buf('c.dmu', B, C).data_ptr(), self.buf('c.dls', B, C).data_ptr()
        cc = sol.constraint_critic
        ch.distributional, ch.deterministic_backup = int(dist), int(sol.deterministic_backup)
        ch.discount, ch.qc_td_bound = sol.discount, sol.qc_td_bound
        ch.lmin, ch.lmax = cc.log_std_min, cc.log_std_max
        ch.log_alpha = sol.log_alpha.data_ptr()
        ch.eps3 = _p(e3)
        ch.dc = ws['c.dm'].data_ptr() if robust else 0
        ch.cost, ch.v = int(self.cost), self.bv.data_ptr()
        ch.seed, ch.ctr = noise.seed, ctr
        ch.loss = loss.data_ptr()
        # per-16-row-tile loss partials (twin 0 | twin 1 | certificate), summed into
        # loss[0] / loss[1] by the weight-gradient launch's extra block
        nt = (B + 15) // 16
        lpart = self.buf('c.lpart', 3 * nt)
        ch.loss_part = lpart.data_ptr()
        # backward: critics (twin) and constraint critic (trunk + heads), each job forming
        # its own output gradients (and loss) from the critic head in-kernel
        # (src/ssac.py:284-456: compute_target, compute_cons_target, both losses)
        heads = [n['cc_trunk'], n['cc_mean']] + ([n['cc_ls']] if dist else [])
        self._run_bwd_multi('c.b' + str(int(dist)), lambda: [
            fill_bwd(heads, [None, ws['c.dmu'], ws['c.dls']][:len(heads)], B, trunk=True, upstream=UPSTREAM_CERT),
            fill_bwd([n['q0'], n['q1']], [ws['c.dq0'], ws['c.dq1']], B, upstream=UPSTREAM_CRITIC)], head=ch)
        tsy = n['cc_trunk'].sy
        items = [(n['q0'], [xs, n['q0'].sy[0], n['q0'].sy[1]], 'c'), (n['q1'], [xs, n['q1'].sy[0], n['q1'].sy[1]], 'c'),
                 (n['cc_trunk'], [xs, tsy[0]], 'cc'), (n['cc_mean'], [tsy[-1], n['cc_mean'].sy[0]], 'cc')]
        if dist:
            items.append((n['cc_ls'], [tsy[-1], n['cc_ls'].sy[0]], 'cc'))
        sq = self._sq('c', ('c', 'cc'))
        used = self._run_wgrad('c.wg' + str(int(dist)) + ('f' if sq else ''), lambda: wgrad_items(items, B, sq),
                               sums=[(lpart[:2 * nt], loss[0]), (lpart[2 * nt:], loss[1])])
        cg = sol.critic_group
        self.dp.sum_(cg.grad)      # the 1/G of the mean rides in the optimizer segments
        crange = cg.span('critic.')
        ccrange = self._alive_span(cg, ['constraint_critic.trunk.', 'constraint_critic.mean_head.'] +
                                   (['constraint_critic.log_std_head.'] if dist else []))
        # two clip norms (critic, constraint critic), one Adam step, grad zeroing, EMA of
        # the whole target group and the packed-mirror refresh: one launch
        tg = sol.critic_target_group
        parts = self._clip_parts(used if sq else None, 'c', ('c', 'cc'),
                                 [cg.grad[s0:s1] for s0, s1 in (crange, ccrange)])
        sc = sol.critic_optimizer.step_scalars()
        mp = cg.pack_map(tg)
        segs = [sol.critic_optimizer.segment(s0, s1, sc, clip=(pt, sol.grad_norm), zero_grad=True,
                                             ema=(tg.data, sol.tau), pack_map=mp, grad_scale=self.dp.scale)
                for (s0, s1), pt in zip((crange, ccrange), parts)]
        lo = 0
        for s0, s1 in sorted((crange, ccrange)) + [(cg.size, cg.size)]:
            if s0 > lo:      # parameters without a gradient (vanilla log-std head): EMA only
                segs.append(ema_segment(cg.data, lo, s0, tg.data, sol.tau, mp))
            lo = max(lo, s1)
        fused_step(segs)
        self._grads_zeroed(cg)
        sol.critic_lr_scheduler.step()
        return loss[0], loss[1]

    def _out_net(self, net, name, B):
        """A no-save view of `net` whose final output lands in buffer `name`."""
        v = Net(net.layers)
        v.sy[-1] = self.buf(name, B, net.dout)
        return v

    # ------------------------------------------------------------------
    def update_actor_and_alpha(self, obs, noise=None):
        """SSAC.update_actor_and_alpha (src/ssac.py:458-527)."""
        B = obs.shape[0]
        self._setup(B)
        self.bs.copy_(obs)
        return self._actor_step(noise)

    def _actor_step(self, noise, f1_done=False):
        sol, n, B, S, A, C = self.sol, self.nets, self.B, self.S, self.A, self.C
        self._ensure_packed()
        self.noise = noise = noise or self.noise
        L = _lib.lib()
        ws = self.ws
        dist = sol.distributional_qc
        qshape = (B,) if C == 1 else (B, C)
        mlp_mult = sol.mlp_multiplier
        e5 = self._eps('e5', noise.std_normal((B, A)))
        k = noise.choice(2)
        if dist:
            noise.randn_like(qshape, used=False)       # Qc(s, a)
            if mlp_mult:
                noise.randn_like(qshape, used=False)   # Qc(s, tanh(mu_safe)) for lambda
        # the cost certificate has no safe-actor loss (src/ssac.py:488-494): no a_safe draw
        cost = self.cost
        e6 = None if cost else self._eps('e6', noise.std_normal((B, A)))
        if dist:
            noise.randn_like(qshape, used=False)
        ctr = noise.next()
        cc = sol.constraint_critic
        xa = self.buf('a.x', B, S)   # the actors' shared input save (the wgrad's first-layer Y of both)
        a, lp, u, e = self.buf('a.a', B, A), self.buf('a.lp', B), self.buf('a.u', B, A), self.buf('a.e', B, A)
        a_s, u_s, e_s, am = self.buf('a.as', B, A), self.buf('a.us', B, A), self.buf('a.es', B, A), \
            self.buf('a.am', B, A)
        # launch 1: actor and safe actor rsample (saves for backward) + fused heads, unless
        # the critic update's forward launch already ran them (early_actor)
        if not f1_done:
            self._run_multi('a.f1' + noise_tag(e5), lambda: self._actor_f1_jobs(e5, e6), ctr)
        # launch 2: Q_k(s, a), Qc(s, a), Qc(s, a_safe) with saves; Qc(s, tanh(mu_safe)) for lam
        qk = n['q0'] if k == 0 else n['q1']
        # lam = multiplier(s, bound) chained behind the bound in the same workgroups (no
        # 'a.mult' launch) when the bound is formed in-kernel
        post = mlp_mult and self._post_mult()

        def ccm():
            d = self._ccb(fill_fwd(self._outs_cc('a.ccm'), [(self.bs, S), (am, A), (None, 0)], B, trunk=True),
                          self.buf('a.sqc', B), dist)
            return with_post(d, self._out_net(n['mult'], 'a.multx', B)) if post else d
        # (job order = workgroup dispatch order: the multiplier's chained job, Q_k, then the
        # certificate jobs measured 86.8 us against 90.9 us for the reverse order
        # (profiles/r05/early_actor/order); m.f2 keeps its chained job first)
        self._run_multi(f'a.f2.{k}{int(mlp_mult)}{int(post)}', lambda: ([ccm()] if mlp_mult else []) + [
            fill_fwd([self._reuse(qk, f'a.q{k}')], [(self.bs, S), (a, A), (None, 0)], B)] + (
            [] if cost else [fill_fwd(self._reuse_cc('a.cc2'), [(self.bs, S), (a_s, A), (None, 0)], B, trunk=True)]) + [
            fill_fwd(self._reuse_cc('a.cc'), [(self.bs, S), (a, A), (None, 0)], B, trunk=True)], ctr)
        if mlp_mult and not post:
            # lam = multiplier(s, max_C Qc_ub(s, tanh(mu_safe)))  (no grad); the bound is formed
            # by the forward launch above
            sqc = self.buf('a.sqc', B)
            self._cc_bound_after('a.ccm', sqc, dist)
            self._run_fwd('a.mult', lambda: fill_fwd([self._out_net(n['mult'], 'a.multx', B)],
                                                     [(self.bs, S), (sqc, 1), (None, 0)], B))
        # The actor losses' output gradients are formed inside the two backward launches
        # (drpo_actor_head_t): w.r.t. Q_k (-1/B) and the constraint critic's heads at (s, a)
        # (lam / B on the max-C bound; lam = MLPMultiplier's output transform of 'a.multx',
        # or the scalar multiplier on clamp(Qc, penalty_lb, penalty_ub), src/ssac.py:474-494)
        # and at (s, a_safe) (1 / B), then the squashed-Gaussian backward of both actors
        # and the alpha-loss sum (src/ssac.py:458-505) -- no separate head launches.
        ah = self.desc.get('a.head')
        if ah is None:
            ah = self.desc['a.head'] = ActorHead()
            ub = float(sol.mlp_multiplier_cfg.upper_bound)
            assert ub > 0 or not mlp_mult, 'MLPMultiplier upper_bound must be positive'
            ah.B, ah.C, ah.A, ah.distributional = B, C, A, int(dist)
            ah.std_ratio, ah.log_std_min, ah.log_std_max = float(cc.std_ratio), float(cc.log_std_min), \
                float(cc.log_std_max)
            ah.lams = ws['a.multx'].data_ptr() if mlp_mult else 0
            ah.lam_upper_bound, ah.fixed_lam = ub, float(sol.fixed_multiplier)
            ah.clamp_lb, ah.clamp_ub = float(sol.penalty_lb), float(sol.penalty_ub)
            ah.u[0], ah.e[0], ah.u[1], ah.e[1] = u.data_ptr(), e.data_ptr(), u_s.data_ptr(), e_s.data_ptr()
            ah.dA[0], ah.dA2[0], ah.dA[1] = self.buf('a.dA', B, A).data_ptr(), self.buf('a.dAc', B, A).data_ptr(), \
                self.buf('a.dAs', B, A).data_ptr()
            ah.logp, ah.log_alpha, ah.lp_scale = lp.data_ptr(), sol.log_alpha.data_ptr(), 1.0 / B
            ah.target_entropy = float(sol.target_entropy)
            ah.alpha_sum = self.alpha_sum.data_ptr() if sol.autotune_alpha else 0
        # dL/da of the actor (Q_k part + certificate part, summed in the squash backward in
        # the reference's order) and of the safe actor: one backward launch
        dA, dAc, dAs = self.buf('a.dA', B, A), self.buf('a.dAc', B, A), self.buf('a.dAs', B, A)
        hv, hv2 = self.nets_view['a.cc'], self.nets_view.get('a.cc2')
        gq, gmu, gls, gmu2, gls2 = (self.buf('a.gq', B), self.buf('a.gmu', B, C), self.buf('a.gls', B, C),
                                    self.buf('a.gmu2', B, C), self.buf('a.gls2', B, C))
        self._run_bwd_multi(f'a.b.{k}{int(dist)}', lambda: [
            fill_bwd(hv if dist else hv[:2], [None, gmu, gls][:3 if dist else 2], B, trunk=True,
                     dx={0: (dAc, S, A, False)}, upstream=UPSTREAM_ACTOR_CC)] + ([] if cost else [
            fill_bwd(hv2 if dist else hv2[:2], [None, gmu2, gls2][:3 if dist else 2], B, trunk=True,
                     dx={0: (dAs, S, A, False)}, upstream=UPSTREAM_SAFE_CC)]) + [
            fill_bwd([self.nets_view[f'a.q{k}']], [gq], B, dx={0: (dA, S, A, False)}, upstream=UPSTREAM_NEG_MEAN)],
            actor=ah)
        draw, draws = self.buf('a.draw', B, 2 * A), self.buf('a.draws', B, 2 * A)
        asum = self.alpha_sum
        self._clean_grads(sol.actor.group)
        if not cost:
            self._clean_grads(sol.actor_safe.group)
        self._run_bwd_multi('a.bpi', lambda: [fill_bwd([n['actor']], [draw], B, upstream=UPSTREAM_SQUASH)] + (
            [] if cost else [fill_bwd([n['safe']], [draws], B, upstream=UPSTREAM_SQUASH_SAFE)]), actor=ah)
        na, ns = n['actor'], n['safe']
        asegs = ('a',) if cost else ('a', 's')
        sq = self._sq('a', asegs)
        used = self._run_wgrad('a.wg' + ('f' if sq else ''),
                               lambda: wgrad_items([(na, [xa, na.sy[0], na.sy[1]], 'a')] + (
                                   [] if cost else [(ns, [xa, ns.sy[0], ns.sy[1]], 's')]), B, sq))
        # d alpha_loss / d log_alpha = -exp(log_alpha) * mean(logp + target_entropy) is formed
        # inside the optimizer launch from the alpha-loss sum (src/ssac.py:498-501); under
        # DP the sum is sum-reduced and divided by G*B rows (same value: log_alpha is
        # replicated). The actors' 1/G rides in their optimizer segments.
        self.dp.sum_(self.actor_xchg)        # actor + safe actor grads + alpha-loss sum: one bucket
        gsc = self.dp.scale
        # actor: clip + Adam + cosine; alpha: Adam (no wd, fixed lr); safe actor: clip + Adam +
        # cosine -- one fused optimizer launch (clip partials from the weight gradients)
        ga, gs = sol.actor.group, sol.actor_safe.group
        pa, *ps = self._clip_parts(used if sq else None, 'a', asegs, [ga.grad, gs.grad][:len(asegs)])
        aopt = sol.alpha_optimizer
        if aopt.tensor is None:
            aopt.tensor = sol.log_alpha.view(1)
        segs = [sol.actor_optimizer.segment(0, ga.size, sol.actor_optimizer.step_scalars(), clip=(pa, sol.grad_norm),
                                            zero_grad=True, pack_map=ga.pack_map(), grad_scale=gsc)]
        # without autotune_alpha the reference's optimizer list is [actor, actor_safe], so
        # its "i == 2" clip / schedule of the safe actor never fires (src/ssac.py:507-527)
        safe_full = sol.autotune_alpha
        if sol.autotune_alpha:
            # the gradient is formed from the summed tile partials (overwritten each step)
            segs.append(aopt.segment(0, 1, aopt.step_scalars(), grad=asum[:1],
                                     grad_from_sum=(asum, B * self.dp.world, (B + 15) // 16),
                                     grad_from_sum_kind=2 if sol.use_log_alpha_loss else 0))
        if not cost:   # the cost certificate's optimizer list is [actor, alpha] (src/ssac.py:509-513)
            segs.append(sol.actor_safe_optimizer.segment(0, gs.size, sol.actor_safe_optimizer.step_scalars(),
                                                         clip=(ps[0], sol.grad_norm) if safe_full else None,
                                                         zero_grad=True, pack_map=gs.pack_map(), grad_scale=gsc))
        fused_step(segs)
        self._grads_zeroed(ga)
        if not cost:
            self._grads_zeroed(gs)
        sol.actor_lr_scheduler.step()
        if safe_full and not cost:
            sol.actor_safe_lr_scheduler.step()

    def _early_actor(self, noise):
        """The actor update's first forward joins the critic update's forward launch:
        production (Philox) noise only -- a recorded tape hands over the actor's draws
        after the critic's."""
        return not getattr(noise, 'parity', False)

    def _actor_f1_jobs(self, e5, e6):
        """The actor update's first forward (src/ssac.py:459-461,489-490): actor and safe
        actor rsample with saves for the backward, and tanh(mu_safe), as multi-job forward
        jobs (launched alone as 'a.f1', or appended to the critic update's 'c.f')."""
        sol, n, B, S, A = self.sol, self.nets, self.B, self.S, self.A
        cost, mlp_mult = self.cost, sol.mlp_multiplier
        xa = self.buf('a.x', B, S)   # the actors' shared input save (the wgrad's first-layer Y of both)
        a, lp, u, e = self.buf('a.a', B, A), self.buf('a.lp', B), self.buf('a.u', B, A), self.buf('a.e', B, A)
        a_s, u_s, e_s, am = self.buf('a.as', B, A), self.buf('a.us', B, A), self.buf('a.es', B, A), \
            self.buf('a.am', B, A)
        # One workgroup runs both policies when their shapes pair (the same input, one
        # saved copy of it). Cost certificate: the safe actor only gives tanh(mu_safe) for the
        # multiplier's input (src/ssac.py:473-478), or nothing without the MLP multiplier.
        if cost:
            return [
                with_head(with_head(fill_fwd([n['actor'], n['safe']], [(self.bs, S), (None, 0), (None, 0)], B,
                                             save_x=xa, pair=True), HEAD_RSAMPLE, A, e5, SITE_PI_RS, a=a, logp=lp, u=u,
                                    e=e),
                          HEAD_MEAN, A, None, 0, amean=am, second=True)] if mlp_mult and pairable(n['actor'], n['safe']) \
                else [with_head(fill_fwd([n['actor']], [(self.bs, S), (None, 0), (None, 0)], B, save_x=xa), HEAD_RSAMPLE,
                                A, e5, SITE_PI_RS, a=a, logp=lp, u=u, e=e)] + (
                    [with_head(fill_fwd([Net(n['safe'].layers)], [(self.bs, S), (None, 0), (None, 0)], B), HEAD_MEAN, A,
                               None, 0, amean=am)] if mlp_mult else [])
        elif pairable(n['actor'], n['safe']):
            return [
                with_head(with_head(fill_fwd([n['actor'], n['safe']], [(self.bs, S), (None, 0), (None, 0)], B,
                                             save_x=xa, pair=True), HEAD_RSAMPLE, A, e5, SITE_PI_RS, a=a, logp=lp, u=u,
                                    e=e),
                          HEAD_RSAMPLE, A, e6, SITE_SAFE_RS, a=a_s, u=u_s, e=e_s, amean=am, second=True)]
        else:
            return [
                with_head(fill_fwd([n['actor']], [(self.bs, S), (None, 0), (None, 0)], B, save_x=xa), HEAD_RSAMPLE,
                          A, e5, SITE_PI_RS, a=a, logp=lp, u=u, e=e),
                with_head(fill_fwd([n['safe']], [(self.bs, S), (None, 0), (None, 0)], B), HEAD_RSAMPLE, A, e6,
                          SITE_SAFE_RS, a=a_s, u=u_s, e=e_s, amean=am)]

    def _alpha_adam(self, grad):
        opt = self.sol.alpha_optimizer
        if opt.tensor is None:
            opt.tensor = self.sol.log_alpha.view(1)
        sc = opt.step_scalars()
        opt.apply(grad, 0, 1, sc)

    # views of nets with separately named save buffers (so passes do not clobber each other)
    def _reuse(self, net, name):
        v = self.nets_view.get(name)
        if v is None:
            v = Net(net.layers, net.grad_layers)
            for l, (_, _, din, dout, act, _) in enumerate(net.layers):
                v.sy[l] = self.buf(f'{name}.sy{l}', self.B, dout)
            self.nets_view[name] = v
        return v

    def _reuse_cc(self, name):
        v = self.nets_view.get(name)
        if v is None:
            v = [self._reuse(x, f'{name}.{i}') for i, x in enumerate(self._cc_nets())]
            self.nets_view[name] = v
        return v

    def _cc_views(self, name):
        v = self.nets_view[name]
        return v[1].sy[-1], v[2].sy[-1]

    def _outs_cc(self, name):
        nets = [Net(x.layers) for x in self._cc_nets()]
        nets[1].sy[-1] = self.buf(f'{name}.mu', self.B, self.C)
        nets[2].sy[-1] = self.buf(f'{name}.ls', self.B, self.C)
        return nets

    # ------------------------------------------------------------------
    def update_multiplier(self, obs, noise=None):
        """SSAC.update_multiplier (src/ssac.py:529-578)."""
        B = obs.shape[0]
        self._setup(B)
        self.bs.copy_(obs)
        return self._mult_step(noise)

    def _mult_step(self, noise):
        sol, n, B, S, A, C = self.sol, self.nets, self.B, self.S, self.A, self.C
        self._ensure_packed()
        self.noise = noise = noise or self.noise
        if not sol.mlp_multiplier:
            return self._scalar_mult_step(noise)
        L = _lib.lib()
        ws = self.ws
        dist = sol.distributional_qc
        qshape = (B,) if C == 1 else (B, C)
        e7 = self._eps('e7', noise.std_normal((B, A)))
        if dist:
            noise.randn_like(qshape, used=False)
            noise.randn_like(qshape, used=False)
        ctr = noise.next()
        a, am = self.buf('m.a', B, A), self.buf('m.am', B, A)
        # launch 1: a ~ pi(s) (rsample) and tanh(mu_safe(s)) via fused heads
        if pairable(n['actor'], n['safe']):
            jobs = lambda: [
                with_head(with_head(fill_fwd([Net(n['actor'].layers), Net(n['safe'].layers)],
                                             [(self.bs, S), (None, 0), (None, 0)], B, pair=True),
                                    HEAD_RSAMPLE, A, e7, SITE_PI_MULT, a=a),
                          HEAD_MEAN, A, None, 0, amean=am, second=True)]
        else:
            jobs = lambda: [
                with_head(fill_fwd([Net(n['actor'].layers)], [(self.bs, S), (None, 0), (None, 0)], B), HEAD_RSAMPLE,
                          A, e7, SITE_PI_MULT, a=a),
                with_head(fill_fwd([Net(n['safe'].layers)], [(self.bs, S), (None, 0), (None, 0)], B), HEAD_MEAN, A,
                          None, 0, amean=am)]
        self._run_multi('m.f1' + noise_tag(e7), jobs, ctr)
        # launch 2: constraint critic at (s, a) and at (s, tanh(mu_safe))
        aqc, sqc = self.buf('m.aqc', B), self.buf('m.sqc', B)
        xm = self.buf('m.x', B, S + 1)
        post = self._post_mult()   # the multiplier chained behind the bound at tanh(mu_safe)

        def ccs():
            d = self._ccb(fill_fwd(self._outs_cc('m.ccs'), [(self.bs, S), (am, A), (None, 0)], B, trunk=True), sqc,
                          dist)
            return with_post(d, n['mult'], xm) if post else d
        self._run_multi(f'm.f2{int(post)}', lambda: [
            ccs(), self._ccb(fill_fwd(self._outs_cc('m.cc'), [(self.bs, S), (a, A), (None, 0)], B, trunk=True), aqc,
                             dist)], ctr)
        self._cc_bound_after('m.cc', aqc, dist)
        self._cc_bound_after('m.ccs', sqc, dist)
        if not post:
            self._run_fwd('m.mult', lambda: fill_fwd([n['mult']], [(self.bs, S), (sqc, 1), (None, 0)], B,
                                                     save_x=xm))
        gx = self.buf('m.gx', B)
        mc = sol.mlp_multiplier_cfg
        _lib.check(L.drpo_multiplier_head(B, n['mult'].sy[-1].data_ptr(), sqc.data_ptr(), aqc.data_ptr(),
                                          float(sol.constraint_threshold), float(sol.penalty_lb),
                                          float(sol.penalty_ub), float(mc.upper_bound), float(sol.lam_epsilon),
                                          gx.data_ptr(), None, _lib.stream()), 'multiplier_head')
        g = sol.multiplier_group
        self._clean_grads(g)
        nm = n['mult']
        self._run_bwd('m.bmult', lambda: fill_bwd([nm], [gx], B))
        sq = self._sq('m', ('m',))
        used = self._run_wgrad('m.wg' + ('f' if sq else ''),
                               lambda: wgrad_items([(nm, [xm, nm.sy[0], nm.sy[1]], 'm')], B, sq))
        self.dp.sum_(g.grad)
        pm, = self._clip_parts(used if sq else None, 'm', ('m',), [g.grad])
        fused_step([sol.multiplier_optimizer.segment(0, g.size, sol.multiplier_optimizer.step_scalars(),
                                                     clip=(pm, sol.grad_norm), zero_grad=True,
                                                     pack_map=g.pack_map(), grad_scale=self.dp.scale)])
        self._grads_zeroed(g)
        sol.multiplier_lr_scheduler.step()

    def _scalar_mult_step(self, noise):
        """Scalar-multiplier branch of SSAC.multiplier_loss / update_multiplier
        (src/ssac.py:529-578 with mlp_multiplier=False): lam_loss = -softplus(m) *
        mean(clamp(Qc(s, a) - threshold, lb, ub)), a ~ pi(s); plain Adam, no clip, no
        schedule. One forward launch, one head launch summing the penalty, and the
        optimizer launch forms d/dm = -sigmoid(m) * sum / rows on the device."""
        sol, n, B, S, A, C = self.sol, self.nets, self.B, self.S, self.A, self.C
        L = _lib.lib()
        ws = self.ws
        dist = sol.distributional_qc
        qshape = (B,) if C == 1 else (B, C)
        e7 = self._eps('e7', noise.std_normal((B, A)))
        if dist:
            noise.randn_like(qshape, used=False)
        ctr = noise.next()
        a = self.buf('m.a', B, A)
        self._run_multi('m.f1s' + noise_tag(e7), lambda: [
            with_head(fill_fwd([Net(n['actor'].layers)], [(self.bs, S), (None, 0), (None, 0)], B), HEAD_RSAMPLE, A,
                      e7, SITE_PI_MULT, a=a)], ctr)
        aqc = self.buf('m.aqc', B)
        self._run_multi('m.f2s', lambda: [
            self._ccb(fill_fwd(self._outs_cc('m.cc'), [(self.bs, S), (a, A), (None, 0)], B, trunk=True), aqc,
                      dist)], ctr)
        self._cc_bound_after('m.cc', aqc, dist)
        psum = self._loss_slots(1)
        _lib.check(L.drpo_multiplier_head(B, None, None, aqc.data_ptr(), float(sol.constraint_threshold),
                                          float(sol.penalty_lb), float(sol.penalty_ub), 0.0, 0.0, None,
                                          psum.data_ptr(), _lib.stream()), 'multiplier_head')
        self.dp.sum_(psum)
        opt = sol.multiplier_optimizer
        fused_step([opt.segment(0, 1, opt.step_scalars(), grad_from_sum=(psum, B * self.dp.world),
                                grad_from_sum_kind=1)])

    # ------------------------------------------------------------------
    def update_solver(self, alg, update_actor, update_multiplier, noise):
        """SMBPO.update_solver (src/smbpo.py:251-279) from the device-resident buffers."""
        sol = self.sol
        B = sol.batch_size
        self._setup(B)
        self.noise = noise
        n_real = int(alg.real_fraction * B)
        rb, vb = alg.replay_buffer._module, alg.virt_buffer._module
        ir = noise.randint(len(rb), n_real)
        iv = noise.randint(None, B - n_real)
        if ir is not None:
            self.ws['idx_r'][:n_real].copy_(torch.from_numpy(ir))
        if iv is not None:
            self.ws['idx_v'][:B - n_real].copy_(torch.from_numpy(iv))
        ctr = noise.next()

        def view(b, dev_len):
            v = BufferView()
            v.s, v.a, v.s2, v.r = b._states.data_ptr(), b._actions.data_ptr(), b._next_states.data_ptr(), \
                b._rewards.data_ptr()
            v.h, v.d, v.v = b._constraint_values.data_ptr(), b._dones.data_ptr(), b._violations.data_ptr()
            v.len = -1 if dev_len else len(b)
            v.ptr_dev = b._pointer.data_ptr()
            v.cap = b.capacity
            return v

        rv, vv = view(rb, False), view(vb, True)
        L = _lib.lib()
        _lib.check(L.drpo_sample_batch(ctypes.byref(rv), ctypes.byref(vv), n_real, B, self.S, self.A, self.Ch,
                                       None if ir is None else self.ws['idx_r'].data_ptr(),
                                       None if iv is None else self.ws['idx_v'].data_ptr(), noise.seed, ctr,
                                       float(alg.reward_scale), float(alg.alive_bonus), float(alg.constraint_scale),
                                       float(alg.constraint_offset), self.bs.data_ptr(), self.ba.data_ptr(),
                                       self.bs2.data_ptr(), self.br.data_ptr(), self.bd.data_ptr(),
                                       self.bv.data_ptr(), self.bh.data_ptr(), _lib.stream()), 'sample_batch')
        early = update_actor and self._early_actor(noise)
        lq, lqc = self._critic_step(noise, early_actor=early)
        if update_actor:
            self._actor_step(noise, f1_done=early)
        if update_multiplier:
            self._mult_step(noise)
        return lq, lqc
