"""Flat, HBM-resident parameter groups with reference-compatible module trees.

Every optimizer group of the reference (critic+constraint critic, actor, safe actor,
multiplier, model ensemble) lives in ONE contiguous fp32 buffer, with matching
flat buffers for gradients and Adam moments. The ``nn.Parameter`` objects the
user sees (and that ``state_dict`` / ``load_state_dict`` touch) are views into
that buffer, laid out exactly like the reference's ``mlp()`` Sequentials
(src/torch_util.py:190-211) so checkpoints keep their key names and shapes.
One flat buffer per group means one kernel for Adam / grad-norm / EMA and one
RCCL bucket per group for data parallelism.

Initialisation replays the reference's CPU-RNG consumption order exactly
(nn.Linear construction + xavier_normal_ / zeros_ from weight_initializer,
src/torch_util.py:146-155; BatchedLinear's (E+1) nn.Linear resets,
src/dynamics.py:26-47), so for a given torch seed the initial weights are
bit-identical to the reference's.
"""
import math

import torch
import torch.nn as nn

ALIGN = 64   # floats: every tensor starts 256-byte aligned (float4 weight loads)


class FlatGroup:
    """Contiguous storage for one parameter group (+ grad / Adam m / v)."""

    def __init__(self, name):
        self.name = name
        self.entries = {}      # name -> (offset, shape)
        self.order = []
        self.size = 0
        self.data = None
        self.grad = None

    def add(self, name, shape):
        n = int(math.prod(shape))
        self.entries[name] = (self.size, tuple(shape))
        self.order.append(name)
        self.size += (n + ALIGN - 1) // ALIGN * ALIGN
        return name

    def allocate(self, device):
        self.data = torch.zeros(self.size, dtype=torch.float32, device=device)
        self.grad = torch.zeros(self.size, dtype=torch.float32, device=device)
        return self

    def view(self, name, buf=None):
        off, shape = self.entries[name]
        n = int(math.prod(shape))
        b = self.data if buf is None else buf
        return b[off:off + n].view(shape)

    def offset(self, name):
        return self.entries[name][0]

    # ---- packed weight mirrors (csrc/pack.hip) ---------------------------------
    def enable_packing(self, layers, transposed=None):
        """layers: [(weight_name, din, dout, nbatch)]. Allocates the forward mirror
        (and the transposed one for trained groups) that every MLP kernel streams."""
        transposed = self.grad is not None if transposed is None else transposed
        self.pk_layers = {}
        off = 0
        for name, din, dout, nb in layers:
            sz = packed_size(din, dout)
            self.pk_layers[name] = (off, sz, din, dout, nb)
            off += sz * nb
        dev = self.data.device
        self.packed = torch.zeros(max(off, 64), dtype=torch.float32, device=dev)
        self.packedT = torch.zeros(max(off, 64), dtype=torch.float32, device=dev) if transposed else None
        self._pk_items = None
        self._pk_ver = None
        return self

    def pview(self, name, transposed=False):
        """[nbatch, packed_size] view of one layer's mirror (row z = member z)."""
        off, sz, din, dout, nb = self.pk_layers[name]
        buf = self.packedT if transposed else self.packed
        return None if buf is None else buf[off:off + sz * nb].view(nb, sz)

    def pack_map(self, target=None):
        """Device-resident drpo_pack_map_t of this group's weight matrices (for the
        fused optimizer step); ``target``: a group of identical layout whose forward
        mirror is refreshed from the EMA'd values."""
        key = None if target is None else target.name
        cache = self.__dict__.setdefault('_pk_maps', {})
        if key in cache:
            return cache[key]
        from ._abi import PackMap
        import ctypes
        mp = PackMap()
        mp.nlayers = len(self.pk_layers)
        assert mp.nlayers <= 16
        for j, (name, (off, sz, din, dout, nb)) in enumerate(self.pk_layers.items()):
            mp.off[j] = self.entries[name][0]
            mp.din[j], mp.dout[j], mp.nbatch[j], mp.poff[j] = din, dout, nb, off
        mp.P = self.packed.data_ptr()
        mp.PT = self.packedT.data_ptr() if self.packedT is not None else 0
        mp.Pt = target.packed.data_ptr() if target is not None else 0
        raw = bytes(mp)
        dev = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.data.device)
        dev.host = mp          # the host copy plans the optimizer's 4x4-block work split
        cache[key] = dev
        return dev

    def move_grad(self, new_grad, *modules):
        """Re-home the flat gradient in ``new_grad`` (e.g. a slice of a shared exchange
        arena), keeping its values; the parameters' .grad views under ``modules`` follow."""
        assert new_grad.numel() == self.size and new_grad.is_contiguous()
        new_grad.copy_(self.grad)
        self.grad = new_grad
        for mod in modules:
            for sub in mod.modules():
                if isinstance(sub, LinearSlot) and sub._group is self:
                    sub.bind_grad()

    def mark_dirty(self):
        """The flat data was written by a kernel (Adam, EMA, a collective)."""
        self._pk_ver = None

    def ensure_packed(self):
        """Refresh the mirrors if the weights changed (torch in-place writes bump the
        shared version counter of the flat buffer and every view of it; kernel writes
        call mark_dirty)."""
        if getattr(self, 'pk_layers', None) is None or self._pk_ver == self.data._version:
            return
        from . import _lib
        from ._abi import PackItem
        if self._pk_items is None:
            items = []
            for name, (off, sz, din, dout, nb) in self.pk_layers.items():
                it = PackItem()
                it.W = self.view(name).data_ptr()
                it.P = self.packed[off:].data_ptr()
                it.PT = self.packedT[off:].data_ptr() if self.packedT is not None else 0
                it.din, it.dout, it.nbatch = din, dout, nb
                it.wstride, it.pstride, it.ptstride = din * dout, sz, sz
                items.append(it)
            self._pk_items = [(PackItem * len(items[i:i + 16]))(*items[i:i + 16]) for i in range(0, len(items), 16)]
        L = _lib.lib()
        for arr in self._pk_items:
            _lib.check(L.drpo_pack_weights(arr, len(arr), _lib.stream()), f'pack {self.name}')
        self._pk_ver = self.data._version

    def span(self, prefix):
        """(start, end) floats covering all entries whose name starts with prefix."""
        offs = [(self.entries[n][0], self.entries[n][0] + int(math.prod(self.entries[n][1])))
                for n in self.order if n.startswith(prefix)]
        return min(o[0] for o in offs), max(o[1] for o in offs)


def packed_size(din, dout):
    """floats in one packed mirror of a [dout][din] weight (== drpo_packed_size)."""
    return ((dout + 15) // 16) * ((din + 15) // 16) * 256


def spec_pack_layers(spec, prefix):
    """[(weight_name, din, dout, nbatch)] of an MLPSpec stored under prefix."""
    return [(f'{prefix}{2 * i}.weight', spec.dims[i], spec.dims[i + 1], spec.E or 1) for i in range(spec.n_layers)]


class LinearSlot(nn.Module):
    """Parameter-holding stand-in for nn.Linear / BatchedLinear (weight [.., out, in], bias [.., out])."""

    def __init__(self, group, prefix):
        super().__init__()
        self._group, self._prefix = group, prefix
        self.weight = nn.Parameter(group.view(prefix + 'weight'), requires_grad=False)
        self.bias = nn.Parameter(group.view(prefix + 'bias'), requires_grad=False)
        self.bind_grad()

    def bind_grad(self):
        """.grad views into the group's flat gradient (again after it moved)."""
        g, p = self._group, self._prefix
        if g.grad is not None:              # target groups (frozen) carry no gradient storage
            self.weight.grad = g.view(p + 'weight', g.grad)
            self.bias.grad = g.view(p + 'bias', g.grad)


class Squeeze(nn.Module):
    def forward(self, x):
        return x.squeeze(1)


_ACT = {'relu': nn.ReLU, 'tanh': nn.Tanh, 'swish': nn.SiLU, 'identity': nn.Identity}


class MLPSpec:
    """Shape of one mlp(): dims, hidden activation, output activation, squeeze."""

    def __init__(self, dims, act='relu', out_act=None, squeeze=False, ensemble=None):
        self.dims, self.act, self.out_act, self.squeeze, self.E = list(dims), act, out_act, squeeze, ensemble

    @property
    def n_layers(self):
        return len(self.dims) - 1

    def layer_shapes(self):
        for i in range(self.n_layers):
            din, dout = self.dims[i], self.dims[i + 1]
            if self.E is None:
                yield 2 * i, (dout, din), (dout,)
            else:
                yield 2 * i, (self.E, dout, din), (self.E, dout)

    def register(self, group, prefix):
        for idx, ws, bs in self.layer_shapes():
            group.add(f'{prefix}{idx}.weight', ws)
            group.add(f'{prefix}{idx}.bias', bs)

    def build(self, group, prefix):
        """nn.Sequential with Linear slots at the reference's indices."""
        layers = []
        for i in range(self.n_layers):
            layers.append(LinearSlot(group, f'{prefix}{2 * i}.'))
            if i < self.n_layers - 1:
                layers.append(_ACT[self.act]())
        if self.out_act is not None:
            layers.append(_ACT[self.out_act]())
        if self.squeeze and self.dims[-1] == 1:
            layers.append(Squeeze())
        return nn.Sequential(*layers)

    def reference_init(self, group, prefix):
        """Consume the CPU generator exactly like mlp(dims, layer_factory) and write the
        resulting weights into the flat group."""
        ws = []
        for i in range(self.n_layers):
            din, dout = self.dims[i], self.dims[i + 1]
            if self.E is None:
                nn.Linear(din, dout)                        # construction-time reset_parameters
                ws.append(torch.empty(dout, din))
            else:
                lin = nn.Linear(din, dout)                  # BatchedLinear.reset_parameters
                for _ in range(self.E):
                    lin.reset_parameters()
                ws.append(torch.empty(self.E, dout, din))
        for i, w in enumerate(ws):                          # net.apply(weight_initializer())
            nn.init.xavier_normal_(w)
            group.view(f'{prefix}{2 * i}.weight').copy_(w)
            group.view(f'{prefix}{2 * i}.bias').zero_()


def layer_views(group, prefix, spec, buf=None):
    """[(W, b)] views for each Linear of an MLP stored under prefix."""
    return [(group.view(f'{prefix}{2 * i}.weight', buf), group.view(f'{prefix}{2 * i}.bias', buf))
            for i in range(spec.n_layers)]
