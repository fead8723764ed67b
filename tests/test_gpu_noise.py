"""Production noise (Philox4x32-10 + Box-Muller on the hardware transcendentals):
the device draws used when no recorded tape is given must be standard normal and
distinct across counters (statistical checks on 2.4M draws)."""
import numpy as np
import pytest
import torch

from drpo_amd import _lib

pytestmark = pytest.mark.gpu


def draws(n, S, seed, ctr):
    L = _lib.lib()
    dev = torch.device('cuda')
    D = torch.zeros(n, S + 1, device=dev)
    LV = torch.zeros(n, S + 1, device=dev)
    s = torch.zeros(n, S, device=dev)
    lo, hi = torch.full((S + 1,), -30., device=dev), torch.full((S + 1,), 30., device=dev)
    s2, r = torch.empty(n, S, device=dev), torch.empty(n, device=dev)
    _lib.check(L.drpo_ens_head(D.data_ptr(), LV.data_ptr(), s.data_ptr(), 0, n, S, 1, lo.data_ptr(), hi.data_ptr(),
                               None, None, seed, ctr, None, None, s2.data_ptr(), r.data_ptr(), _lib.stream()))
    torch.cuda.synchronize()
    # lv = clamp(0) -> std = sqrt(exp(lv))
    lv = 30 - np.log1p(np.exp(30.0))
    lv = -30 + np.log1p(np.exp(lv + 30))
    return torch.cat([s2, r[:, None]], 1).cpu().numpy().astype(np.float64) / np.sqrt(np.exp(lv))


def test_device_normals_are_standard():
    z = draws(200000, 11, 123, 7).ravel()
    assert abs(z.mean()) < 5e-3
    assert abs(z.std() - 1) < 5e-3
    kurt = ((z - z.mean()) ** 4).mean() / z.var() ** 2
    assert abs(kurt - 3) < 0.05
    # tails: P(|z| > 3) = 0.0027
    assert abs((np.abs(z) > 3).mean() - 0.0027) < 4e-4


def test_device_normals_decorrelated_across_counters_and_seeds():
    a, b, c = draws(50000, 11, 123, 7).ravel(), draws(50000, 11, 123, 8).ravel(), draws(50000, 11, 124, 7).ravel()
    assert abs(np.corrcoef(a, b)[0, 1]) < 0.01
    assert abs(np.corrcoef(a, c)[0, 1]) < 0.01
    assert not np.array_equal(a, b)
    # adjacent draws within a stream are uncorrelated
    assert abs(np.corrcoef(a[:-1], a[1:])[0, 1]) < 0.01


@pytest.mark.parametrize('use_idx', [False, True])
def test_fit_gather_steps_matches_per_step_gathers(use_idx):
    """drpo_ens_gather_steps (the fit's chunked minibatch gather) writes, for step k,
    exactly what drpo_ens_gather writes with Philox counter ctr + k (or idx rows
    [k*rows, (k+1)*rows)), from a wrapped circular replay (pointer past capacity)."""
    L = _lib.lib()
    dev = torch.device('cuda')
    S, A, cap, rows, steps = 5, 2, 1000, 96, 4
    g = torch.Generator().manual_seed(5)
    bs, ba, bs2, br = (torch.randn(cap, S, generator=g), torch.randn(cap, A, generator=g),
                       torch.randn(cap, S, generator=g), torch.randn(cap, generator=g))
    bs, ba, bs2, br = bs.to(dev), ba.to(dev), bs2.to(dev), br.to(dev)
    ptr = torch.tensor([1234], dtype=torch.int64, device=dev)           # wrapped: 234 is the oldest row
    idx = torch.randint(0, cap, (steps * rows,), generator=g).to(dev) if use_idx else None
    seed, ctr = 0x1234567, 40

    def run(n_steps, c, idx_ptr, out):
        _lib.check(L.drpo_ens_gather_steps(bs.data_ptr(), ba.data_ptr(), bs2.data_ptr(), br.data_ptr(), 0,
                                           ptr.data_ptr(), cap, rows, n_steps, idx_ptr, seed, c, S, A,
                                           out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(),
                                           _lib.stream()))

    big = (torch.full((steps * rows, S), -7., device=dev), torch.full((steps * rows, A), -7., device=dev),
           torch.full((steps * rows, S + 1), -7., device=dev))
    run(steps, ctr, None if idx is None else idx.data_ptr(), big)
    for k in range(steps):
        one = (torch.empty(rows, S, device=dev), torch.empty(rows, A, device=dev), torch.empty(rows, S + 1, device=dev))
        _lib.check(L.drpo_ens_gather(bs.data_ptr(), ba.data_ptr(), bs2.data_ptr(), br.data_ptr(), 0, ptr.data_ptr(),
                                     cap, rows, None if idx is None else idx[k * rows:].data_ptr(), seed,
                                     0 if idx is not None else ctr + k, S, A, one[0].data_ptr(), one[1].data_ptr(),
                                     one[2].data_ptr(), _lib.stream()))
        for a, b in zip(big, one):
            assert torch.equal(a[k * rows:(k + 1) * rows], b)
    # the draws differ between steps (distinct counters)
    if idx is None:
        assert not torch.equal(big[0][:rows], big[0][rows:2 * rows])
