"""RNG tape recorder used ONLY by tests/golden/make_golden.py (build container).

While active, it wraps the random sources the reference's hot path draws from
(see SURVEY.md §3.3 for the order):

  torch.normal(loc, scale)      -> Normal.sample        (src/squashed_gaussian.py via torch.distributions)
  Tensor.normal_()              -> Normal.rsample        (_standard_normal)
  torch.randn_like(x)           -> src/dynamics.py:202, src/ssac.py:80
  torch.randint(...)            -> src/sampling.py:148, src/dynamics.py:166,174
  random.choice(seq)            -> src/dynamics.py:199, src/ssac.py:43
  np.random.choice(...)         -> src/torch_util.py:44
  torch.rand(...)               -> UniformPolicy.act (src/policy.py:43-47, warm-up)

Every wrapper leaves the generator consumption and the returned value exactly
as the original (the reference runs unmodified); it only records the standard
normal draw (``eps``), the integer draw, or the chosen index, in call order.
"""
import random

import numpy as np
import torch

_orig = {}


class Tape:
    def __init__(self):
        self.entries = []  # list of (kind, np.ndarray)
        self.active = False

    # ---- wrappers -------------------------------------------------------
    def _normal(self, *args, **kwargs):
        if len(args) == 2 and torch.is_tensor(args[0]) and torch.is_tensor(args[1]) and not kwargs:
            loc, scale = args
            shape = torch.broadcast_shapes(loc.shape, scale.shape)
            state = torch.get_rng_state()
            eps = torch.randn(shape, dtype=loc.dtype)
            torch.set_rng_state(state)
            out = _orig['normal'](loc, scale)
            # CPU normal(mean,std) == normal_(0,1) * std + mean: verify we captured eps exactly
            assert torch.equal(eps * scale + loc, out), 'eps capture mismatch'
            self.entries.append(('normal', eps.numpy().copy()))
            return out
        return _orig['normal'](*args, **kwargs)

    def _normal_(self, t, *args, **kwargs):
        out = _orig['normal_'](t, *args, **kwargs)
        self.entries.append(('normal_', out.detach().numpy().copy()))
        return out

    def _randn_like(self, x, *args, **kwargs):
        out = _orig['randn_like'](x, *args, **kwargs)
        self.entries.append(('randn_like', out.detach().numpy().copy()))
        return out

    def _randint(self, *args, **kwargs):
        out = _orig['randint'](*args, **kwargs)
        self.entries.append(('randint', out.numpy().copy()))
        return out

    def _rand(self, *args, **kwargs):
        out = _orig['rand'](*args, **kwargs)
        self.entries.append(('rand', out.detach().numpy().copy()))
        return out

    def _choice(self, seq):
        idx = _orig['choice'](range(len(seq)))
        self.entries.append(('choice', np.array(idx, dtype=np.int64)))
        return seq[idx]

    def _np_choice(self, *args, **kwargs):
        out = _orig['np_choice'](*args, **kwargs)
        self.entries.append(('np_choice', np.asarray(out).copy()))
        return out

    def __enter__(self):
        _orig.update(normal=torch.normal, normal_=torch.Tensor.normal_, randn_like=torch.randn_like,
                     randint=torch.randint, choice=random.choice, np_choice=np.random.choice,
                     rand=torch.rand)
        torch.normal = self._normal
        torch.Tensor.normal_ = lambda t, *a, **k: self._normal_(t, *a, **k)
        torch.randn_like = self._randn_like
        torch.randint = self._randint
        torch.rand = self._rand
        random.choice = self._choice
        np.random.choice = self._np_choice
        self.active = True
        return self

    def __exit__(self, *exc):
        torch.normal = _orig['normal']
        torch.Tensor.normal_ = _orig['normal_']
        torch.randn_like = _orig['randn_like']
        torch.randint = _orig['randint']
        torch.rand = _orig['rand']
        random.choice = _orig['choice']
        np.random.choice = _orig['np_choice']
        self.active = False

    def to_npz_dict(self, prefix='tape'):
        d = {f'{prefix}_n': np.array(len(self.entries))}
        for i, (kind, arr) in enumerate(self.entries):
            d[f'{prefix}_{i:04d}_{kind}'] = arr
        return d
