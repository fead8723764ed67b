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
