"""Dynamics-ensemble engine: BatchedGaussianEnsemble's forward / sample / loss / fit
(src/dynamics.py:112-253) as HIP launches over the model's flat HBM group.

Every pass is one fused MLP launch over all members (grid.z = member; weights are
the [E, out, in] BatchedLinear layout, so member z reads W + z*out*in) around
small row-wise kernels (csrc/ensemble.hip):

  forward     drpo_mlp_forward (trunk + diff head + log-var head in one launch)
              -> drpo_ens_head (residual mean, soft log-var clamp [, sample])
  fit step    drpo_ens_gather -> forward (saving activations) -> drpo_ens_loss
              (NLL + bound term + output grads) -> drpo_mlp_backward (heads into
              the shared trunk) -> drpo_mlp_wgrad (all 6 layers x E members, one
              launch) -> drpo_adam over the whole group
  holdout     gather -> forward with member stride 0 (the reference's
              .repeat(E, 1) without the copy) -> drpo_ens_loss (no grads)

The per-step ``loss.item()`` of the reference is deferred: losses land in a device
array that is read once at the end of fit (same returned list of floats).
"""
import ctypes

import numpy as np
import torch

from . import _lib
from .optim import fused_step
from .rng import DeviceNoise
from .sac_step import ACT_ID, Net, fill_bwd, fill_fwd
from ._abi import EnsReduce, EnsUpstream, WgradItem


# Forward: one workgroup per (row tile, head) when the plain grid (16-row tiles x
# members) would leave most of the 256 CUs idle. The trunk is recomputed per head
# (1.33x the forward FLOPs) but each workgroup's serial chain shortens from 5 to 3
# dense layers: fit forward 28.8 -> 20.1 us at E=7, b=256 (csrc/mlp.hip, split_heads).
# Backward: the same split -- one workgroup per (row tile, head), each forming the NLL
# gradient of its head in-kernel (drpo_mlp_backward_ens) and backing its share through
# the trunk -- leaves the trunk dZ as two terms (dz + dz2). The weight-gradient launch
# takes both terms as ONE item (drpo_wgrad_item_t.dz2: the product (dz + dz2)^T y reads
# the trunk activations once; round 2's two-item form re-read them and was rejected).
SPLIT_HEADS_MAX_TILES = 256


def split_heads(n, Z):
    return (n + 15) // 16 * Z <= SPLIT_HEADS_MAX_TILES


def ens_fused_shapes(nets, S1):
    """The shapes drpo_mlp_backward_ens accepts (csrc/mlp.hip): both heads
    [H -> 200|256 -> S+1] with the same hidden width and activation and an identity
    output layer, S+1 <= 64, and every trunk layer at most 256 wide."""
    h1, h2 = nets[1].layers, nets[2].layers
    if len(h1) != 2 or len(h2) != 2 or S1 > 64:
        return False
    (_, _, _, hid1, act1, _), (_, _, _, hid2, act2, _) = h1[0], h2[0]
    if hid1 not in (200, 256) or hid1 != hid2 or act1 != act2:
        return False
    if h1[1][3] != S1 or h2[1][3] != S1 or h1[1][4] != 0 or h2[1][4] != 0:
        return False
    return all(din <= 256 and dout <= 256 for (_, _, din, dout, _, _) in nets[0].layers)


def ens_fb_shapes(nets, S, A):
    """The shapes drpo_ens_fit_fb takes (csrc/fit.hip: the fit step's forward, NLL and
    backward-data in one launch): trunk [S+A <= 64 -> H -> H], heads [H -> H -> S+1 <= 16],
    swish hidden layers, identity outputs, H = 200 | 256 (the reference default:
    src/dynamics.py:59-61,85-86, hidden_dim=200, trunk_layers=2, head_hidden_layers=1)."""
    if len(nets) != 3 or S + A > 64 or S + 1 > 16:
        return False
    sw = ACT_ID['swish']
    t = nets[0].layers
    if len(t) != 2:
        return False
    H = t[1][3]
    if H not in (200, 256) or t[0][3] != H or t[0][4] != sw or t[1][4] != sw:
        return False
    for h in (nets[1].layers, nets[2].layers):
        if len(h) != 2 or h[0][2] != H or h[0][3] != H or h[0][4] != sw or h[1][3] != S + 1 or h[1][4] != 0:
            return False
    return True


class EnsembleEngine:
    def __init__(self, model):
        self.m = model
        # single-process fit: Adam (+ mirror refresh) fused into the weight-gradient launch
        # (drpo_mlp_wgrad_adam; bitwise the same step as drpo_optim_step). The three switches
        # below are the production dispatch; the bitwise / parity tests turn them off to run
        # the launches each fusion replaced as their reference
        # (tests/test_gpu_configs.py::test_fit_fused_adam_matches_separate_step,
        # ::test_fit_fb_matches_two_launches).
        self.fused_adam = True
        self.split_bwd = True     # one backward workgroup per (row tile, head); False: paired heads
        self.fit_fb_enabled = True   # forward + NLL + backward-data as one launch (drpo_ens_fit_fb)
        self.ws = {}
        self.wg_ws = {}
        self.noise = None
        self.dev = model.group.data.device
        from .distributed import GradReducer
        self.dp = GradReducer()

    # ------------------------------------------------------------------ helpers
    def buf(self, name, *shape, dtype=torch.float32):
        t = self.ws.get(name)
        if t is None or t.numel() < int(np.prod(shape)) or t.dtype != dtype:
            t = torch.empty(int(np.prod(shape)), dtype=dtype, device=self.dev)
            self.ws[name] = t
        return t[:int(np.prod(shape))].view(*shape)

    def _noise(self, noise):
        if noise is not None:
            return noise
        if self.noise is None:
            self.noise = DeviceNoise(torch.initial_seed() ^ 0x5EED0DE1)
        return self.noise

    def _specs(self):
        m = self.m
        return (('trunk.', m.trunk_spec), ('diff_head.', m.diff_spec), ('log_var_head.', m.logvar_spec))

    def _nets(self, member=None, grads=False, z0=0):
        """Kernel views of the trunk and both heads: one member (``member``) or the
        members from ``z0`` on (member stride; z0 > 0 for an ensemble shard)."""
        g = self.m.group
        nets, strides = [], []
        for prefix, spec in self._specs():
            lay, gl, st = [], [], []
            for i in range(spec.n_layers):
                key = f'{prefix}{2 * i}.weight'
                W, WT, b = g.pview(key), g.pview(key, True), g.view(f'{prefix}{2 * i}.bias')
                din, dout = spec.dims[i], spec.dims[i + 1]
                act = spec.act if i < spec.n_layers - 1 else spec.out_act
                if member is not None:
                    W, WT, b = W[member], WT[member], b[member]
                    st.append((0, 0))
                else:          # packed-mirror stride per member, bias stride
                    st.append((W.shape[1], dout))
                    W, WT, b = W[z0], WT[z0], b[z0]
                lay.append((W, b, din, dout, ACT_ID[act], WT))
                if grads:
                    gl.append((g.view(f'{prefix}{2 * i}.weight', g.grad)[z0],
                               g.view(f'{prefix}{2 * i}.bias', g.grad)[z0]))
            nets.append(Net(lay, gl if grads else None))
            strides.append(st)
        return nets, strides

    # ------------------------------------------------------------------ forward
    def _forward_desc(self, s, a, n, Z, s_zs, a_zs, member=None, tag='f', save=False, z0=0):
        """Descriptor of one fused ensemble forward (raw head outputs D, LVR [Z*n, S+1]);
        with save=True the activations needed for the backward pass are kept."""
        m = self.m
        S, A = m.state_dim, m.action_dim
        S1 = S + 1
        m.group.ensure_packed()
        nets, strides = self._nets(member, grads=save, z0=z0)
        rows = Z * n
        split = split_heads(n, Z)
        if save:
            for j, net in enumerate(nets):
                for l, (_, _, din, dout, act, _) in enumerate(net.layers):
                    net.sy[l] = self.buf(f'{tag}.sy{j}{l}', rows, dout)
                    net.sz[l] = self.buf(f'{tag}.sz{j}{l}', rows, dout) if act == ACT_ID['swish'] else None
                    net.dz[l] = self.buf(f'{tag}.dz{j}{l}', rows, dout)
                    if j == 0 and self.split_bwd and split:
                        net.dz2[l] = self.buf(f'{tag}.dzb{l}', rows, dout)
            save_x = self.buf(f'{tag}.x', rows, S + A)
        else:
            save_x = None
            nets[1].sy[-1] = self.buf(f'{tag}.D', rows, S1)
            nets[2].sy[-1] = self.buf(f'{tag}.L', rows, S1)
        norm = m.state_normalizer
        d = fill_fwd(nets, [(s, S), (a, A)], n, trunk=True, save_x=save_x, norm=(norm.mean, norm.std), nbatch=Z,
                     wstride=strides, sstride=[s_zs, a_zs, 0], split_heads=split)
        return d, nets, strides, save_x

    def _forward(self, s, a, n, Z, s_zs, a_zs, member=None, tag='f', save=False, z0=0):
        d, nets, strides, save_x = self._forward_desc(s, a, n, Z, s_zs, a_zs, member, tag, save, z0)
        _lib.check(_lib.lib().drpo_mlp_forward(ctypes.byref(d), _lib.stream()), 'ensemble forward')
        return nets, strides, save_x

    def _head(self, D, LVR, s, s_zs, n, Zo, zsel=None, eps=None, noise=None, outputs=('mu', 'lv'), out=None):
        m, L = self.m, _lib.lib()
        S = m.state_dim
        if out is not None:
            outputs = ()
        out = {} if out is None else out
        if 'mu' in outputs:
            out['mu'] = torch.empty(Zo, n, S + 1, device=self.dev)
            out['lv'] = torch.empty(Zo, n, S + 1, device=self.dev)
        if 's2' in outputs:
            out['s2'] = torch.empty(Zo, n, S, device=self.dev)
            out['r'] = torch.empty(Zo, n, device=self.dev)
        seed, ctr = (0, 0)
        if 's2' in out and eps is None:
            nz = self._noise(noise)
            seed, ctr = nz.seed, nz.next()
        zs = None
        if zsel is not None:
            zs = torch.tensor(list(zsel), dtype=torch.int32, device=self.dev)
        _lib.check(L.drpo_ens_head(_lib.ptr(D), _lib.ptr(LVR), _lib.ptr(s), s_zs, n, S, Zo, _lib.ptr(m.min_log_var),
                                   _lib.ptr(m.max_log_var), _lib.ptr(zs), _lib.ptr(eps), seed, ctr,
                                   _lib.ptr(out.get('mu')), _lib.ptr(out.get('lv')), _lib.ptr(out.get('s2')),
                                   _lib.ptr(out.get('r')), _lib.stream()), 'ens_head')
        return out

    def _prep(self, *xs):
        _lib.require_device(self.m.group.data, *xs)
        return [x.contiguous().float() for x in xs]

    def forward1(self, s, a, index):
        s, a = self._prep(s, a)
        n = s.shape[0]
        nets, _, _ = self._forward(s, a, n, 1, 0, 0, member=int(index))
        o = self._head(nets[1].sy[-1], nets[2].sy[-1], s, 0, n, 1)
        return o['mu'][0], o['lv'][0]

    def forward_all(self, s, a):
        """s [E|1, n, S], a [E|1, n, A] (leading 1 = shared rows, stride 0)."""
        s, a = self._prep(s, a)
        E = self.m.ensemble_size
        n = s.shape[-2]
        s_zs = 0 if s.dim() == 2 or s.shape[0] == 1 else n * s.shape[-1]
        a_zs = 0 if a.dim() == 2 or a.shape[0] == 1 else n * a.shape[-1]
        if s.dim() == 3:
            assert s.shape[0] in (1, E) and a.shape[0] in (1, E)
        nets, _, _ = self._forward(s, a, n, E, s_zs, a_zs)
        o = self._head(nets[1].sy[-1], nets[2].sy[-1], s, s_zs, n, E)
        return o['mu'], o['lv']

    def sample(self, s, a, index, noise, eps=None, out=None, tag='f'):
        """sample (src/dynamics.py:198-203) for member ``index``. eps: recorded draws
        (device tensor) or None (tape / Philox); out: optional {'s2', 'r'} buffers."""
        s, a = self._prep(s, a)
        n, S = s.shape
        if eps is None and noise is not None and noise.parity:
            eps = torch.from_numpy(noise.randn_like((n, S + 1))).to(self.dev)
        nets, _, _ = self._forward(s, a, n, 1, 0, 0, member=int(index), tag=tag)
        o = self._head(nets[1].sy[-1], nets[2].sy[-1], s, 0, n, 1, eps=eps, noise=noise, outputs=('s2',), out=out)
        return o['s2'].reshape(n, S), o['r'].reshape(n)

    def elite_samples(self, s, a, elites, noise):
        s, a = self._prep(s, a)
        n, S = s.shape
        E = self.m.ensemble_size
        eps = None
        if noise is not None and noise.parity:
            eps = torch.from_numpy(noise.randn_like((len(elites), n, S + 1))).to(self.dev)
        nets, _, _ = self._forward(s, a, n, E, 0, 0)
        o = self._head(nets[1].sy[-1], nets[2].sy[-1], s, 0, n, len(elites), zsel=elites, eps=eps, noise=noise,
                       outputs=('s2',))
        return o['s2'], o['r']

    # ------------------------------------------------------------------ loss / grads
    def _loss_ws(self, tag, b, Z):
        """Partial-sum workspace of drpo_ens_loss."""
        nb = int(_lib.lib().drpo_ens_loss_workspace_size(b, self.m.state_dim, Z))
        key = f'{tag}.lossws'
        t = self.ws.get(key)
        if t is None or t.numel() < nb:
            t = torch.zeros(nb, dtype=torch.uint8, device=self.dev)
            self.ws[key] = t
        return t

    def _loss_args(self, nets, s, s_zs, t, t_zs, b, Z, grads, gscale=None, loss_out=None, tag='f', bound=True):
        m = self.m
        S = m.state_dim
        S1 = S + 1
        g = m.group
        mse = self.buf(f'{tag}.mse', Z)
        D, LVR = nets[1].sy[-1], nets[2].sy[-1]
        gD = gL = gmin = gmax = None
        if grads:
            gD, gL = self.buf(f'{tag}.gD', Z * b, S1), self.buf(f'{tag}.gL', Z * b, S1)
            gmin, gmax = g.view('min_log_var', g.grad), g.view('max_log_var', g.grad)
        args = [_lib.ptr(D), _lib.ptr(LVR), _lib.ptr(s), s_zs, _lib.ptr(t), t_zs, b, S, Z, _lib.ptr(m.min_log_var),
                _lib.ptr(m.max_log_var), float(m.log_var_bound_weight) if bound else 0.0, _lib.ptr(gscale),
                _lib.ptr(mse), _lib.ptr(loss_out), _lib.ptr(gD), _lib.ptr(gL), _lib.ptr(gmin), _lib.ptr(gmax),
                _lib.ptr(self._loss_ws(tag, b, Z))]
        return args, mse, gD, gL

    def _loss(self, nets, s, s_zs, t, t_zs, b, Z, grads, gscale=None, loss_out=None, tag='f', bound=True):
        args, mse, gD, gL = self._loss_args(nets, s, s_zs, t, t_zs, b, Z, grads, gscale, loss_out, tag, bound)
        _lib.check(_lib.lib().drpo_ens_loss(*args, _lib.stream()), 'ens_loss')
        return mse, gD, gL

    def _backward_descs(self, nets, strides, save_x, gD, gL, b, Z):
        """Backward-data descriptor and the weight-gradient items: (desc, [(items, n)]).
        Split heads (EnsembleEngine.split_bwd) leave the trunk dZ as two terms, which the trunk
        layers' items carry as dz + dz2."""
        split = nets[0].dz2[0] is not None
        d = fill_bwd(nets, [None, gD, gL], b, trunk=True, nbatch=Z, wstride=strides, split_heads=split)
        items = []
        trunk_out = nets[0].sy[-1]
        for j, net in enumerate(nets):
            ins = [save_x if j == 0 else trunk_out] + [net.sy[l] for l in range(len(net.layers) - 1)]
            for l, (W, bb, din, dout, act, _) in enumerate(net.layers):
                gW, gb = net.grad_layers[l]
                it = WgradItem()
                it.dz, it.y, it.gW, it.gb = net.dz[l].data_ptr(), ins[l].data_ptr(), gW.data_ptr(), gb.data_ptr()
                it.dz2 = 0 if net.dz2[l] is None else net.dz2[l].data_ptr()
                it.dout, it.din, it.rows, it.nbatch = dout, din, b, Z
                it.zstride, it.ystride, it.gwstride, it.gbstride = b * dout, b * din, dout * din, dout
                items.append(it)
        return d, [((WgradItem * len(items))(*items), len(items))]

    def _wgrad_ws(self, key, arr, n):
        """Per-call-site weight-gradient workspace (sized once per descriptor array)."""
        c = self.wg_ws.get(key)
        if c is not None and c[0] is arr:
            return c[1]
        from .sac_step import wgrad_workspace
        ws = wgrad_workspace(self.ws, f'{key}.wgws', arr, n, self.dev)
        self.wg_ws[key] = (arr, ws)
        return ws

    def _wgrad(self, key, launches, red=None, stream=None):
        L = _lib.lib()
        stream = _lib.stream() if stream is None else stream
        for k, (arr, n) in enumerate(launches):
            ws = self._wgrad_ws(f'{key}{k}', arr, n)
            if k == 0 and red is not None:
                _lib.check(L.drpo_mlp_wgrad_reduce(arr, n, ctypes.byref(red), ws.data_ptr(), ws.numel(), stream),
                           'ensemble wgrad')
            else:
                _lib.check(L.drpo_mlp_wgrad(arr, n, ws.data_ptr(), ws.numel(), stream), 'ensemble wgrad')

    def _backward(self, nets, strides, save_x, gD, gL, b, Z):
        L = _lib.lib()
        d, launches = self._backward_descs(nets, strides, save_x, gD, gL, b, Z)
        _lib.check(L.drpo_mlp_backward(ctypes.byref(d), _lib.stream()), 'ensemble backward')
        self._wgrad('cl', launches)

    def compute_loss_value(self, s, a, t, with_grads=False, gscale=None):
        """compute_loss on explicit rows (truncated to a multiple of E); returns a 0-d device
        loss, optionally accumulating the gradients into the group's grad."""
        s, a, t = self._prep(s, a, t)
        E = self.m.ensemble_size
        n = len(t) - len(t) % E
        b = n // E
        assert b >= 1, f'compute_loss needs at least {E} rows'
        S, A = self.m.state_dim, self.m.action_dim
        s, a, t = s[:n], a[:n], t[:n]
        loss = torch.empty((), device=self.dev)
        nets, strides, save_x = self._forward(s, a, b, E, b * S, b * A, tag='cl', save=True)
        mse, gD, gL = self._loss(nets, s, b * S, t, b * (S + 1), b, E, with_grads, gscale=gscale, loss_out=loss,
                                 tag='cl')
        if with_grads:
            self._backward(nets, strides, save_x, gD, gL, b, E)
        return loss

    # ------------------------------------------------------------------ fit
    def fit(self, buffer, steps, noise=None):
        """fit(steps=) (src/dynamics.py:155-183). Under data parallelism the members are
        sharded over the ranks (distributed.MemberShard) unless dp_mode='batch', in which
        case every rank fits all members on its own draw and the gradients are averaged."""
        from .distributed import member_sharding
        m, L = self.m, _lib.lib()
        nz = self._noise(noise)
        rb = getattr(buffer, '_module', buffer)
        _lib.require_device(m.group.data, rb._states)
        n = len(rb)
        S, A = m.state_dim, m.action_dim
        S1 = S + 1
        sh = member_sharding(m)
        # Normalizer over the chronological states (physical rows [0, n) hold the same set)
        m.state_normalizer.fit(rb._states[:n])
        if sh is not None:       # one normalizer for the whole ensemble (rank 0's replay)
            sh.broadcast_(m.state_normalizer.mean, m.state_normalizer.std)
        elif self.dp.active:     # batch DP: replicas must normalise alike too
            self.dp.broadcast_(m.state_normalizer.mean, m.state_normalizer.std)
        E, b = m.ensemble_size, m.batch_size
        z0, Z = (sh.z0, sh.count) if sh is not None else (0, E)
        rows = Z * b
        xs, xa, xt = self.buf('fit.s', rows, S), self.buf('fit.a', rows, A), self.buf('fit.t', rows, S1)
        losses = torch.empty(max(steps, 1), device=self.dev)
        ptr_dev = rb._pointer if rb._host_ptr is None else None
        ptr_host = rb._host_ptr if rb._host_ptr is not None else 0

        def gather(count, out, full=None):
            # parity mode: the reference's randint over all E*b rows, this shard's slice
            idx = nz.randint(n, full or count) if nz.parity else None
            if idx is not None and full:
                idx = idx[z0 * b:z0 * b + count]
            idx_t = None if idx is None else torch.from_numpy(np.ascontiguousarray(idx)).to(self.dev)
            ctr = 0 if nz.parity else nz.next()
            _lib.check(L.drpo_ens_gather(_lib.ptr(rb._states), _lib.ptr(rb._actions), _lib.ptr(rb._next_states),
                                         _lib.ptr(rb._rewards), ptr_host, _lib.ptr(ptr_dev), rb.capacity, count,
                                         _lib.ptr(idx_t), nz.seed, ctr, S, A, _lib.ptr(out[0]), _lib.ptr(out[1]),
                                         _lib.ptr(out[2]), _lib.stream()), 'ens_gather')

        g = m.group
        g.grad.zero_()
        if sh is None:   # batch DP: the gradient is sum-reduced, the optimizer applies 1/G
            segs = [m.optimizer.segment(0, g.size, (0.0, 1.0), zero_grad=True, pack_map=g.pack_map(),
                                        grad_scale=self.dp.scale)]
        else:
            ranges = self._shard_ranges(z0, Z)
            lo, hi = g.offset('min_log_var'), g.offset('max_log_var') + S1
            bounds_grad = g.grad[lo:hi]
            pmap = g.pack_map()
            segs = [m.optimizer.segment(a, c, (0.0, 1.0), zero_grad=True, pack_map=pmap) for a, c in ranges]
        # the whole step is built once (descriptors point at fixed workspaces); per step
        # only the minibatch indices / Philox counter, the loss slot and Adam's bias-
        # corrected step sizes change
        from ._abi import OptimSeg
        seg_arr = [(OptimSeg * len(segs[k:k + 8]))(*segs[k:k + 8]) for k in range(0, len(segs), 8)]
        fd, nets, strides, save_x = self._forward_desc(xs, xa, b, Z, b * S, b * A, tag='fit', save=True, z0=z0)
        largs, _, gD, gL = self._loss_args(nets, xs, b * S, xt, b * S1, b, Z, True, loss_out=losses[0:1], tag='fit',
                                           bound=sh is None or sh.rank == 0)
        bd, wl = self._backward_descs(nets, strides, save_x, gD, gL, b, Z)
        # the NLL loss rides in the backward launch (its output gradients formed in-kernel)
        # and its reduction in the weight-gradient launch: forward, backward, wgrad, Adam.
        # That needs the shapes drpo_mlp_backward_ens takes (the reference default:
        # head_hidden_layers=1, 200-wide); other shapes keep the separate loss launch.
        fused = ens_fused_shapes(nets, S1)
        bd.upstream = 3 if fused else 0   # DRPO_UPSTREAM_ENS
        # the reference default shapes at split-heads grids: forward + NLL + backward-data
        # as ONE launch per (row tile, head) (drpo_ens_fit_fb)
        fb = self.fit_fb_enabled and fused and bool(bd.split_heads) and ens_fb_shapes(nets, S, A)
        self.fit_fb = fb
        up = EnsUpstream()
        up.D, up.LVR = nets[1].sy[-1].data_ptr(), nets[2].sy[-1].data_ptr()
        up.s_zstride, up.t_zstride, up.b, up.S, up.Z = b * S, b * S1, b, S, Z
        up.minlv, up.maxlv = m.min_log_var.data_ptr(), m.max_log_var.data_ptr()
        up.part = self._loss_ws('fit', b, Z).data_ptr()
        red_in = EnsReduce()
        red_in.weight = float(m.log_var_bound_weight) if (sh is None or sh.rank == 0) else 0.0
        red_in.mse = self.buf('fit.mse', Z).data_ptr()
        red_in.gmin = g.view('min_log_var', g.grad).data_ptr()
        red_in.gmax = g.view('max_log_var', g.grad).data_ptr()
        red = EnsReduce()
        full = E * b if sh is not None else rows
        idx_all = None
        if nz.parity and steps > 0:
            draws = [np.asarray(nz.randint(n, full))[z0 * b:z0 * b + rows] for _ in range(steps)]
            idx_all = torch.from_numpy(np.ascontiguousarray(np.stack(draws), dtype=np.int64)).to(self.dev)
        stream = _lib.stream()
        # Adam fused into the weight-gradient launch: single process, whole group, no clip
        fuse = self.fused_adam and fused and sh is None and not self.dp.active and len(wl) == 1
        # Member shard: the rank-local members take the same fused weight-
        # gradient + Adam launch (their tiles of the group's pack map); only the shared
        # log-var bounds' 2(S+1) gradients leave the step. Their reduction runs as its own
        # one-block launch on a side stream as soon as the backward has written the NLL
        # partials; the side stream then sum-all-reduces them (the step's ONE collective)
        # and steps the bounds, overlapped with the members' launch on the main stream.
        # The next step's backward (which reads the bounds and rewrites the partials)
        # waits for it.
        # (a member shard and batch DP exclude each other: member_sharding() is None under
        # dp_mode='batch', and no shard path sum-reduces the member gradients)
        assert sh is None or getattr(m, 'dp_mode', 'auto') != 'batch'
        fuse_sh = self.fused_adam and fused and sh is not None and len(wl) == 1
        self.fit_path = 'fused' if fuse else ('fused-shard' if fuse_sh else 'separate')   # (tests, probes)
        if fuse or fuse_sh:
            from ._abi import WgradAdam
            opt = m.optimizer
            opt._ensure_state()
            pm = g.pack_map()
            ad = WgradAdam()
            ad.g, ad.p, ad.m, ad.v = g.grad.data_ptr(), g.data.data_ptr(), opt.m.data_ptr(), opt.v.data_ptr()
            ad.beta1, ad.beta2 = opt.betas
            ad.eps, ad.weight_decay = opt.eps, opt.weight_decay
            ad.map, ad.map_host = pm.data_ptr(), ctypes.addressof(pm.host)
            warr, wn = wl[0]
            wws = self._wgrad_ws('fit0', warr, wn)
        if fuse_sh:
            bseg = (OptimSeg * 1)(m.optimizer.segment(lo, hi, (0.0, 1.0), zero_grad=True))
            side = self.__dict__.setdefault('_side', torch.cuda.Stream(device=self.dev))
            if getattr(self, '_side_evs', None) is None:   # fence-free library events (csrc/core.hip)
                self._side_evs = []
                for _ in range(2):
                    e = ctypes.c_void_p()
                    _lib.check(L.drpo_event_create(ctypes.byref(e)), 'event_create')
                    self._side_evs.append(e)
            ev_bwd, ev_done = self._side_evs
            main_s = stream
            side_s = ctypes.c_void_p(side.cuda_stream)
            pending = False
        gargs = [_lib.ptr(rb._states), _lib.ptr(rb._actions), _lib.ptr(rb._next_states), _lib.ptr(rb._rewards),
                 ptr_host, _lib.ptr(ptr_dev), rb.capacity, rows]
        loss_base = losses.data_ptr()
        # The minibatches of a chunk of steps are gathered in ONE launch (the replay is
        # not written during the fit); the step's forward / loss descriptors are pointed
        # at its slice. Chunks of <= 64 MB of gathered rows.
        W = 2 * S + A + 1
        chunk = max(1, min(steps, (64 << 20) // (4 * W * max(rows, 1))))
        cs, ca, ct = (self.buf('fit.s_all', chunk * rows, S), self.buf('fit.a_all', chunk * rows, A),
                      self.buf('fit.t_all', chunk * rows, S1))
        for i in range(steps):
            k = i % chunk
            if k == 0:
                nc = min(chunk, steps - i)
                if idx_all is not None:
                    idx, ctr = ctypes.c_void_p(idx_all.data_ptr() + 8 * rows * i), 0
                else:   # the counters the per-step draws would take: ctr, ctr + 1, ...
                    idx, ctr = None, nz.next()
                    for _ in range(nc - 1):
                        nz.next()
                _lib.check(L.drpo_ens_gather_steps(*gargs, nc, idx, nz.seed, ctr, S, A, _lib.ptr(cs), _lib.ptr(ca),
                                                   _lib.ptr(ct), stream), 'ens_gather')
            fd.src[0], fd.src[1] = cs.data_ptr() + 4 * k * rows * S, ca.data_ptr() + 4 * k * rows * A
            up.s, up.t = fd.src[0], ct.data_ptr() + 4 * k * rows * S1
            red_in.loss = loss_base + 4 * i
            if not fb:
                _lib.check(L.drpo_mlp_forward(ctypes.byref(fd), stream), 'ensemble forward')
            if fuse_sh and pending:           # the previous step's bounds are stepped
                _lib.check(L.drpo_stream_wait_event(main_s, ev_done), 'stream_wait_event')
            if fb:
                _lib.check(L.drpo_ens_fit_fb(ctypes.byref(fd), ctypes.byref(bd), ctypes.byref(up),
                                             ctypes.byref(red_in), ctypes.byref(red), stream), 'ensemble fit fwd+bwd')
            elif fused:
                _lib.check(L.drpo_mlp_backward_ens(ctypes.byref(bd), ctypes.byref(up), ctypes.byref(red_in),
                                                   ctypes.byref(red), stream), 'ensemble backward')
            else:
                largs[2], largs[4], largs[14] = ctypes.c_void_p(up.s), ctypes.c_void_p(up.t), \
                    ctypes.c_void_p(red_in.loss)
                _lib.check(L.drpo_ens_loss_partials(*largs, ctypes.byref(red), stream), 'ens_loss')
                _lib.check(L.drpo_mlp_backward(ctypes.byref(bd), stream), 'ensemble backward')
            if fuse:
                # weight gradients + the NLL reduction + Adam + mirror refresh: one launch
                ad.lr_over_bc1, ad.bc2_sqrt = m.optimizer.step_scalars()
                _lib.check(L.drpo_mlp_wgrad_adam(warr, wn, ctypes.byref(red), ctypes.byref(ad), wws.data_ptr(),
                                                 wws.numel(), stream), 'ensemble wgrad + adam')
                continue
            if fuse_sh:
                lr_bc1, bc2 = m.optimizer.step_scalars()
                _lib.check(L.drpo_event_record(ev_bwd, main_s), 'event_record')
                _lib.check(L.drpo_stream_wait_event(side_s, ev_bwd), 'stream_wait_event')
                _lib.check(L.drpo_ens_loss_reduce(ctypes.byref(red), side_s), 'ens_loss_reduce')
                with torch.cuda.stream(side):      # the collective on the side stream
                    sh.sum_(bounds_grad)
                bseg[0].lr_over_bc1, bseg[0].bc2_sqrt = lr_bc1, bc2
                _lib.check(L.drpo_optim_step(bseg, 1, side_s), 'optim_step (log-var bounds)')
                _lib.check(L.drpo_event_record(ev_done, side_s), 'event_record')
                pending = True
                ad.lr_over_bc1, ad.bc2_sqrt = lr_bc1, bc2
                _lib.check(L.drpo_mlp_wgrad_adam(warr, wn, None, ctypes.byref(ad), wws.data_ptr(), wws.numel(),
                                                 stream), 'ensemble wgrad + adam (member shard)')
                continue
            # the loss reduction rides as the last workgroup of the wgrad launch
            self._wgrad('fit', wl, red, stream)
            if sh is None:
                self.dp.sum_(g.grad)
            else:
                sh.sum_(bounds_grad)      # shared log-var bounds: the sum over all members
            # Adam + grad zeroing + packed-mirror refresh in one launch
            lr_bc1, bc2 = m.optimizer.step_scalars()
            for arr in seg_arr:
                for k in range(len(arr)):
                    arr[k].lr_over_bc1, arr[k].bc2_sqrt = lr_bc1, bc2
                _lib.check(L.drpo_optim_step(arr, len(arr), stream), 'optim_step')
        if fuse_sh and pending:
            _lib.check(L.drpo_stream_wait_event(main_s, ev_done), 'stream_wait_event')
        # holdout: the same rows for every member (src/dynamics.py:175-183)
        hb = m.holdout_size
        assert hb == b, 'reference asserts holdout_size == batch_size (src/dynamics.py:177)'
        hs, ha, ht = self.buf('ho.s', hb, S), self.buf('ho.a', hb, A), self.buf('ho.t', hb, S1)
        gather(hb, (hs, ha, ht))
        if sh is not None:
            sh.broadcast_(hs, ha, ht)
        nets, _, _ = self._forward(hs, ha, hb, Z, 0, 0, tag='ho', z0=z0)
        mse, _, _ = self._loss(nets, hs, 0, ht, 0, hb, Z, False, tag='ho')
        if sh is None:
            self.dp.mean_(mse)       # identical elites on every rank
        else:
            mse = sh.merge_members(mse, torch.zeros(E, device=self.dev))
            sh.sum_(losses)          # per-step loss = sum of the shards' member terms
            self._gather_members(sh)
        mse_h = mse.tolist()
        m.holdout_losses = mse_h
        m._elite_inds = [int(i) for i in np.argsort(np.asarray(mse_h, np.float32), kind='stable')[:m.num_elites]]
        return [float(x) for x in losses[:steps].tolist()]

    def _shard_ranges(self, z0, Z):
        """Flat-group element ranges of members [z0, z0+Z) of every layer, plus the
        shared log-var bounds (the Adam segments of a member shard)."""
        g, out = self.m.group, []
        for prefix, spec in self._specs():
            for i in range(spec.n_layers):
                for key in (f'{prefix}{2 * i}.weight', f'{prefix}{2 * i}.bias'):
                    off, shape = g.entries[key]
                    per = int(np.prod(shape[1:]))
                    out.append((off + z0 * per, off + (z0 + Z) * per))
        S1 = self.m.state_dim + 1
        out.append((g.offset('min_log_var'), g.offset('max_log_var') + S1))
        return out

    def _gather_members(self, sh):
        """Every member's weights on every rank after a sharded fit."""
        g = self.m.group
        for prefix, spec in self._specs():
            for i in range(spec.n_layers):
                for key in (f'{prefix}{2 * i}.weight', f'{prefix}{2 * i}.bias'):
                    sh.gather_members_(g.view(key))
        g.mark_dirty()

    def _gather_buffer(self, rb, count, idx_t, seed, ctr, out):
        m, L = self.m, _lib.lib()
        _lib.check(L.drpo_ens_gather(_lib.ptr(rb._states), _lib.ptr(rb._actions), _lib.ptr(rb._next_states),
                                     _lib.ptr(rb._rewards), rb.pointer, None, rb.capacity, count, _lib.ptr(idx_t),
                                     seed, ctr, m.state_dim, m.action_dim, _lib.ptr(out[0]), _lib.ptr(out[1]),
                                     _lib.ptr(out[2]), _lib.stream()), 'ens_gather')

    def fit_epochs(self, buffer, epochs, max_grad_norm=None, post_epoch_callback=None, post_step_callback=None,
                   progress_bar=False, verbose=False):
        """fit(epochs=) == epochal_training over E*epochs epochs of randperm minibatches of
        E*batch_size rows (src/dynamics.py:185-190, src/train.py:58-100). randperm uses the
        CPU generator like the reference; the minibatch rows are gathered on the device."""
        from .optim import grad_sumsq
        m = self.m
        rb = getattr(buffer, '_module', buffer)
        _lib.require_device(m.group.data, rb._states)
        n = len(rb)
        S, A = m.state_dim, m.action_dim
        m.state_normalizer.fit(rb._states[:n])
        # the same data-parallel contract as fit(steps=): one normalizer (rank 0's) on
        # every replica, gradients sum-reduced with the 1/G in the optimizer
        self.dp.broadcast_(m.state_normalizer.mean, m.state_normalizer.std)
        E, tb = m.ensemble_size, m.total_batch_size
        n_batches = -(-n // tb)
        losses = []
        for epoch in range(E * epochs):
            perm = torch.randperm(n).to(self.dev)
            ep = torch.empty(n_batches, device=self.dev)
            for bi in range(n_batches):
                idx = perm[bi * tb:min(n, (bi + 1) * tb)]
                cnt = len(idx)
                xs, xa, xt = self.buf('ep.s', cnt, S), self.buf('ep.a', cnt, A), self.buf('ep.t', cnt, S + 1)
                self._gather_buffer(rb, cnt, idx, 0, 0, (xs, xa, xt))
                m.group.grad.zero_()
                ep_i = ep[bi:bi + 1].view(())
                loss = self.compute_loss_value(xs, xa, xt, with_grads=True)
                ep_i.copy_(loss)
                self.dp.sum_(m.group.grad)
                # Adam (clipped on the reduced gradient's norm when asked) with the DP 1/G
                # applied to the gradient and its norm inside the step
                clip = None
                if max_grad_norm is not None:
                    clip = (grad_sumsq(m.group.grad), max_grad_norm)
                sc = m.optimizer.step_scalars()
                fused_step([m.optimizer.segment(0, m.group.size, sc, clip=clip, pack_map=m.group.pack_map(),
                                                grad_scale=self.dp.scale)])
                if post_step_callback is not None:
                    post_step_callback(epoch, bi, n_batches)
            losses.append(float(np.mean(ep.tolist())))
            if post_epoch_callback is not None:
                post_epoch_callback(epoch)
        return losses


class EnsembleLoss(torch.autograd.Function):
    """compute_loss as a differentiable 0-d tensor for external training loops
    (src/train.py:58-69 epochal_training: loss.backward(); optimizer.step()).
    backward() re-runs the fused forward with gradients (scaled by the incoming
    grad) and accumulates into the flat group's grad (= every parameter's .grad)."""

    @staticmethod
    def forward(ctx, anchor, engine, s, a, t):
        ctx.engine, ctx.rows = engine, (s, a, t)
        return engine.compute_loss_value(s, a, t, with_grads=False)

    @staticmethod
    def backward(ctx, g):
        s, a, t = ctx.rows
        ctx.engine.compute_loss_value(s, a, t, with_grads=True, gscale=g.detach().contiguous().float())
        return None, None, None, None, None
