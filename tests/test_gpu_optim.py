"""drpo_optim_step (csrc/optim.hip): the fused optimizer launch with the 4x4-block
work split over weight matrices (segments carrying a host copy of their pack map)
against the flat 4-element split of the same launch and against a float64 torch
restatement of torch.optim.Adam's single-tensor update with coupled weight decay
(the reference's optimizers, src/ssac.py:507-527, src/dynamics.py:155-183) and
clip_grad_norm_'s coefficient.

Checked: Adam state and parameters, gradient zeroing, the EMA target
(src/torch_util.py:223-226), and the packed mirrors (forward, transposed, target
forward) equal a fresh drpo_pack_weights of the updated weights -- bitwise, since
both splits run the same per-element arithmetic. Shapes cover din % 4 != 0 (14),
dout % 4 != 0 (13, 1), ensemble members (nbatch 3), a segment that starts inside a
matrix's member range (flat fallback for the partial member) and non-matrix
entries (biases, a [5] vector)."""
import ctypes

import numpy as np
import pytest
import torch

import drpo_amd  # noqa: F401
from drpo_amd.optim import Adam, ema_segment, fused_step, grad_sumsq
from drpo_amd.params import FlatGroup

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda')
LAYERS = [('a.weight', 14, 200, 3), ('b.weight', 200, 13, 3), ('c.weight', 256, 256, 1), ('d.weight', 256, 1, 1)]


def make_group(name, seed, transposed=True, grads=True):
    g = FlatGroup(name)
    for wname, din, dout, nb in LAYERS:
        g.add(wname, (nb, dout, din) if nb > 1 else (dout, din))
        g.add(wname.replace('weight', 'bias'), (nb, dout) if nb > 1 else (dout,))
    g.add('lv', (5,))
    g.allocate(DEV)
    gen = torch.Generator(device='cpu').manual_seed(seed)
    g.data.copy_(torch.randn(g.size, generator=gen))
    if grads:
        g.grad.copy_(torch.randn(g.size, generator=gen) * 0.1)
    else:
        g.grad = None
    g.enable_packing([(n, din, dout, nb) for n, din, dout, nb in LAYERS], transposed=transposed)
    g.ensure_packed()
    return g


def run(block, clip, ema, seg_range=None):
    g = make_group('g', 1)
    t = make_group('t', 2, transposed=False, grads=False) if ema else None
    opt = Adam(g, lr=3e-3, weight_decay=1e-4)
    opt._ensure_state()
    gen = torch.Generator(device='cpu').manual_seed(3)
    opt.m.copy_(torch.randn(g.size, generator=gen) * 0.01)
    opt.v.copy_(torch.rand(g.size, generator=gen) * 0.01)
    g0 = dict(p=g.data.clone(), g=g.grad.clone(), m=opt.m.clone(), v=opt.v.clone(),
              t=t.data.clone() if ema else None)
    pm = g.pack_map(t)
    if not block:
        pm = pm.clone()         # a device map without the host copy: the flat split
    s0, s1 = seg_range or (0, g.size)
    part = grad_sumsq(g.grad[s0:s1]) if clip else None
    sc = opt.step_scalars()
    segs = [opt.segment(s0, s1, sc, clip=(part, 0.5) if clip else None, zero_grad=True,
                        ema=(t.data, 0.01) if ema else None, pack_map=pm)]
    if ema:   # EMA (and mirror refresh) of the parameters outside the Adam segment
        segs += [ema_segment(g.data, a, b, t.data, 0.01, pm) for a, b in ((0, s0), (s1, g.size)) if b > a]
    fused_step(segs)
    torch.cuda.synchronize()
    return g, t, opt, g0, sc, (s0, s1)


def reference(g0, sc, clip, rng, ema):
    s0, s1 = rng
    p, gr, m, v = (g0[k].double().cpu().clone() for k in 'pgmv')
    gs = gr[s0:s1]
    coef = 1.0
    if clip:
        coef = min(1.0, 0.5 / (float(gs.float().pow(2).sum()) ** 0.5 + 1e-6))
    ge = gs * coef + 1e-4 * p[s0:s1]
    m[s0:s1] = m[s0:s1] + (ge - m[s0:s1]) * (1 - 0.9)
    v[s0:s1] = v[s0:s1] * 0.999 + (1 - 0.999) * ge * ge
    p[s0:s1] = p[s0:s1] - sc[0] * (m[s0:s1] / (v[s0:s1].sqrt() / sc[1] + 1e-8))
    t = None
    if ema:
        t = g0['t'].double().cpu().clone()
        t = 0.01 * p + 0.99 * t
    return p, m, v, t


@pytest.mark.parametrize('clip,ema,partial', [(False, False, False), (True, True, False), (True, False, True),
                                              (False, True, True)])
def test_block_split_matches_flat_split_and_reference(clip, ema, partial):
    rng = None
    if partial:
        # start inside matrix 'a' (member 1 of 3, mid-row) and end inside matrix 'c'
        g = make_group('probe', 1)
        rng = (g.offset('a.weight') + 200 * 14 + 37, g.offset('c.weight') + 256 * 100 + 5)
    gb, tb, ob, g0, sc, r = run(True, clip, ema, rng)
    gf, tf, of, _, _, _ = run(False, clip, ema, rng)
    # same per-element arithmetic in both splits: bitwise
    assert torch.equal(gb.data, gf.data)
    assert torch.equal(ob.m, of.m) and torch.equal(ob.v, of.v)
    s0, s1 = r
    assert int((gb.grad[s0:s1] != 0).sum()) == 0           # zeroed
    assert torch.equal(gb.grad[:s0], g0['g'][:s0]) and torch.equal(gb.grad[s1:], g0['g'][s1:])
    if ema:
        assert torch.equal(tb.data, tf.data)
    # mirrors == a fresh pack of the updated weights
    for grp in ([gb] + ([tb] if ema else [])):
        P, PT = grp.packed.clone(), None if grp.packedT is None else grp.packedT.clone()
        grp.mark_dirty()
        grp._pk_ver = None
        grp.ensure_packed()
        torch.cuda.synchronize()
        assert torch.equal(P, grp.packed), f'{grp.name}: forward mirror'
        if PT is not None:
            assert torch.equal(PT, grp.packedT), f'{grp.name}: transposed mirror'
    # float64 torch restatement
    p, m, v, t = reference(g0, sc, clip, r, ema)
    for got, ref, what in ((gb.data, p, 'p'), (ob.m, m, 'm'), (ob.v, v, 'v')) + (((tb.data, t, 't'),) if ema else ()):
        err = (got.double().cpu() - ref).abs()
        tol = 2e-6 * ref.abs() + 1e-7
        assert bool((err <= tol).all()), f'{what}: max err {float(err.max())}'
