"""drpo_mlp_wgrad (csrc/wgrad.hip): grouped weight gradients gW += dZ^T Y, gb +=
colsum(dZ) for every layer of a group in one launch, against a float64 torch
reference of the same products (the autograd of nn.Linear / BatchedLinear,
src/dynamics.py:26-52, src/torch_util.py:190-211).

Covers every tile shape (64 / 16 wide on either side), widths that are not
multiples of 4 or 16, row counts that leave partial k-groups and partial row chunks,
ensemble batches (nbatch > 1), split-K over row chunks (the last-arriver combine),
the per-tile clip partials (sum of squares of the finished gradient), accumulation
into a non-zero gradient, bitwise determinism across launches and the workspace
being left zeroed. Tolerance (fp32 MFMA vs float64): |d| <= 1e-5 * sqrt(rows) *
max|ref| + 1e-5 * |ref|."""
import ctypes

import numpy as np
import pytest
import torch

import drpo_amd  # noqa: F401
from drpo_amd import _lib
from drpo_amd._abi import WgradItem

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda')


def make_items(shapes, rows, nbatch=1, seed=0, accumulate=False):
    g = torch.Generator().manual_seed(seed)
    out = []
    for dout, din in shapes:
        dz = torch.randn(nbatch, rows, dout, generator=g)
        y = torch.randn(nbatch, rows, din, generator=g)
        gW0 = torch.randn(nbatch, dout, din, generator=g) if accumulate else torch.zeros(nbatch, dout, din)
        gb0 = torch.randn(nbatch, dout, generator=g) if accumulate else torch.zeros(nbatch, dout)
        out.append(dict(dz=dz.to(DEV), y=y.to(DEV), gW=gW0.to(DEV), gb=gb0.to(DEV), gW0=gW0, gb0=gb0,
                        dout=dout, din=din))
    return out


def run(items, rows, nbatch, ws=None, sq=None):
    L = _lib.lib()
    arr = (WgradItem * len(items))()
    off = 0
    for k, d in enumerate(items):
        it = arr[k]
        it.dz, it.y, it.gW, it.gb = d['dz'].data_ptr(), d['y'].data_ptr(), d['gW'].data_ptr(), d['gb'].data_ptr()
        it.dout, it.din, it.rows, it.nbatch = d['dout'], d['din'], rows, nbatch
        it.zstride, it.ystride, it.gwstride, it.gbstride = rows * d['dout'], rows * d['din'], d['dout'] * d['din'], \
            d['dout']
        if sq is not None:
            it.sq, it.sq_off = sq.data_ptr(), off
            d['sq_off'] = off
            d['ntiles'] = L.drpo_mlp_wgrad_tiles(ctypes.byref(it))
            off += d['ntiles']
    need = L.drpo_mlp_wgrad_workspace_size(arr, len(items))
    if ws is None:
        ws = torch.zeros(max(need, 256), dtype=torch.uint8, device=DEV)
    _lib.check(L.drpo_mlp_wgrad(arr, len(items), ws.data_ptr(), ws.numel(), _lib.stream()), 'wgrad')
    return ws


def reference(d):
    dz, y = d['dz'].double().cpu(), d['y'].double().cpu()
    gW = d['gW0'].double() + torch.einsum('zro,zri->zoi', dz, y)
    gb = d['gb0'].double() + dz.sum(1)
    return gW, gb


def check(d, rows):
    gW, gb = reference(d)
    scale = 1e-5 * np.sqrt(rows) * max(float(gW.abs().max()), 1.0)
    for got, ref, what in ((d['gW'], gW, 'gW'), (d['gb'], gb, 'gb')):
        err = (got.double().cpu() - ref).abs()
        tol = scale + 1e-5 * ref.abs()
        assert bool((err <= tol).all()), f'{what} {d["dout"]}x{d["din"]}: max err {float(err.max())}'
    return gW, gb


# (dout, din) per item: 64x64 tiles, 16-wide outputs (critic / head output layers),
# 16-wide inputs (S+A input layers), both narrow, widths not a multiple of 4 / 16
SHAPES = [(256, 256), (1, 256), (2, 256), (256, 14), (200, 200), (13, 200), (200, 14), (4, 4), (256, 53), (53, 256),
          (7, 13)]


@pytest.mark.parametrize('rows', [1, 37, 256, 1000, 4096])
def test_wgrad_shapes_and_rows(rows):
    items = make_items(SHAPES, rows, seed=rows)
    sq = torch.full((4096,), -1.0, device=DEV)
    run(items, rows, 1, sq=sq)
    torch.cuda.synchronize()
    for d in items:
        gW, gb = check(d, rows)
        # clip partials: sum of squares of the finished gradient, per tile (bias once per o-tile)
        parts = sq[d['sq_off']:d['sq_off'] + d['ntiles']].double().cpu()
        want = float((gW ** 2).sum() + (gb ** 2).sum())
        assert abs(float(parts.sum()) - want) <= 1e-4 * want + 1e-6, (d['dout'], d['din'], float(parts.sum()), want)


@pytest.mark.parametrize('rows,nbatch', [(256, 7), (256, 32), (100, 3), (2048, 2)])
def test_wgrad_ensemble_batches(rows, nbatch):
    shapes = [(200, 14), (200, 200), (200, 200), (13, 200), (200, 200), (13, 200)]
    items = make_items(shapes, rows, nbatch=nbatch, seed=nbatch)
    run(items, rows, nbatch)
    torch.cuda.synchronize()
    for d in items:
        check(d, rows)


def test_wgrad_accumulates_is_deterministic_and_leaves_workspace_zeroed():
    rows = 4096   # several row chunks per tile: the last-arriver combine
    items = make_items([(256, 256), (2, 256), (256, 14)], rows, seed=5, accumulate=True)
    base = [(d['gW'].clone(), d['gb'].clone()) for d in items]
    ws = run(items, rows, 1)
    torch.cuda.synchronize()
    for d in items:
        check(d, rows)
    first = [(d['gW'].clone(), d['gb'].clone()) for d in items]
    # the counters are back to zero (the slabs may hold data): a second launch on the same
    # workspace from the same start gives bitwise the same gradient
    for d, (w, b) in zip(items, base):
        d['gW'].copy_(w)
        d['gb'].copy_(b)
    run(items, rows, 1, ws=ws)
    torch.cuda.synchronize()
    for d, (w, b) in zip(items, first):
        assert torch.equal(d['gW'], w) and torch.equal(d['gb'], b)
    ntiles = 16 + 4 + 4     # arrival counters of the three items (first bytes of the workspace)
    assert int(ws[:4 * ntiles].view(torch.int32).abs().sum()) == 0


def test_wgrad_rejects_shared_gradient_and_small_workspace():
    rows = 64
    items = make_items([(16, 16)], rows)
    L = _lib.lib()
    arr = (WgradItem * 2)()
    for k in range(2):
        d = items[0]
        it = arr[k]
        it.dz, it.y, it.gW, it.gb = d['dz'].data_ptr(), d['y'].data_ptr(), d['gW'].data_ptr(), d['gb'].data_ptr()
        it.dout, it.din, it.rows, it.nbatch = 16, 16, rows, 1
        it.zstride, it.ystride, it.gwstride, it.gbstride = rows * 16, rows * 16, 256, 16
    ws = torch.zeros(1 << 20, dtype=torch.uint8, device=DEV)
    assert L.drpo_mlp_wgrad(arr, 2, ws.data_ptr(), ws.numel(), _lib.stream()) != 0
    big = make_items([(256, 256)], 4096)
    run(big, 4096, 1)          # sized workspace: fine
    arr1 = (WgradItem * 1)()
    d = big[0]
    it = arr1[0]
    it.dz, it.y, it.gW, it.gb = d['dz'].data_ptr(), d['y'].data_ptr(), d['gW'].data_ptr(), d['gb'].data_ptr()
    it.dout, it.din, it.rows, it.nbatch = 256, 256, 4096, 1
    it.zstride, it.ystride, it.gwstride, it.gbstride = 4096 * 256, 4096 * 256, 65536, 256
    assert L.drpo_mlp_wgrad(arr1, 1, ws.data_ptr(), 16, _lib.stream()) != 0


@pytest.mark.parametrize('rows', [37, 1792, 4096])
def test_wgrad_second_dz_term(rows):
    """drpo_wgrad_item_t.dz2 (the split-heads fit backward's trunk dZ = dz + dz2): the
    product is (dz + dz2)^T y and the bias colsum(dz + dz2), for 64-, 16- and odd-width
    tiles, ensemble batches and several row chunks."""
    L = _lib.lib()
    nb = 3
    shapes = [(200, 200), (200, 14), (13, 200)]
    items = make_items(shapes, rows, nbatch=nb, seed=rows + 7)
    g = torch.Generator().manual_seed(rows)
    arr = (WgradItem * len(items))()
    for k, d in enumerate(items):
        d['dz2'] = torch.randn(nb, rows, d['dout'], generator=g).to(DEV)
        it = arr[k]
        it.dz, it.y, it.gW, it.gb = d['dz'].data_ptr(), d['y'].data_ptr(), d['gW'].data_ptr(), d['gb'].data_ptr()
        it.dz2 = d['dz2'].data_ptr()
        it.dout, it.din, it.rows, it.nbatch = d['dout'], d['din'], rows, nb
        it.zstride, it.ystride, it.gwstride, it.gbstride = rows * d['dout'], rows * d['din'], d['dout'] * d['din'], \
            d['dout']
    need = L.drpo_mlp_wgrad_workspace_size(arr, len(items))
    ws = torch.zeros(max(need, 256), dtype=torch.uint8, device=DEV)
    _lib.check(L.drpo_mlp_wgrad(arr, len(items), ws.data_ptr(), ws.numel(), _lib.stream()), 'wgrad')
    torch.cuda.synchronize()
    for d in items:
        dz = (d['dz'] + d['dz2']).double().cpu()
        y = d['y'].double().cpu()
        gW = torch.einsum('zro,zri->zoi', dz, y)
        gb = dz.sum(1)
        scale = 1e-5 * np.sqrt(rows) * max(float(gW.abs().max()), 1.0)
        for got, ref, what in ((d['gW'], gW, 'gW'), (d['gb'], gb, 'gb')):
            err = (got.double().cpu() - ref).abs()
            assert bool((err <= scale + 1e-5 * ref.abs()).all()), f'{what} {d["dout"]}x{d["din"]}: {float(err.max())}'
