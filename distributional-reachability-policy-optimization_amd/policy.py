"""Tanh-squashed diagonal Gaussian policy (src/policy.py:61-100, src/squashed_gaussian.py).

The MLP S->H..->2A (ReLU) lives in a flat parameter group; ``act`` runs the fused
HIP MLP forward + squashed-Gaussian head (see ops.py)."""
import numpy as np
import torch

from .params import FlatGroup, MLPSpec
from .torch_util import Module


class SquashedGaussian(torch.distributions.transformed_distribution.TransformedDistribution):
    """src/squashed_gaussian.py:7-16 (Normal pushed through TanhTransform(cache_size=1))."""

    def __init__(self, loc, scale, validate_args=None):
        from torch.distributions import Normal
        from torch.distributions.transforms import TanhTransform
        super().__init__(Normal(loc, scale), TanhTransform(cache_size=1), validate_args=validate_args)

    @property
    def mean(self):
        mu = self.base_dist.loc
        for t in self.transforms:
            mu = t(mu)
        return mu


class SquashedGaussianPolicy(Module):
    def __init__(self, state_dim, action_dim, hidden_dim=256, hidden_layers=2, group=None, prefix='net.',
                 log_std_bounds=(-6, 4), std_multiplier=1.0):
        super().__init__()
        self.state_dim, self.action_dim = state_dim, action_dim
        self.spec = MLPSpec([state_dim, *([hidden_dim] * hidden_layers), 2 * action_dim], 'relu')
        self.log_std_bounds = log_std_bounds
        self.std_multiplier = std_multiplier
        assert tuple(log_std_bounds) == (-6, 4) and std_multiplier == 1.0, \
            'the fused head implements the reference defaults log_std_bounds=(-6,4), std_multiplier=1'
        self.group = group
        self.prefix = prefix

    @classmethod
    def create(cls, state_dim, action_dim, hidden_dim, hidden_layers, name, device, init=True):
        g = FlatGroup(name)
        pol = cls(state_dim, action_dim, hidden_dim, hidden_layers, group=g)
        pol.spec.register(g, 'net.')
        g.allocate('cpu')
        if init:
            pol.spec.reference_init(g, 'net.')
        g.data = g.data.to(device)
        g.grad = g.grad.to(device)
        from .params import spec_pack_layers
        g.enable_packing(spec_pack_layers(pol.spec, 'net.'))
        pol.net = pol.spec.build(g, 'net.')
        return pol

    def layers(self, buf=None):
        from .params import layer_views
        return layer_views(self.group, 'net.', self.spec, buf)

    def act(self, states, eval, noise=None):
        """TorchPolicy.act (src/policy.py:76-79): fused MLP + squashed-Gaussian head."""
        from . import ops
        return ops.policy_act(self, states, eval, noise)

    def distr(self, states):
        """Independent(SquashedGaussian(mu, std), 1) (src/policy.py:69-70,88-97); loc/scale
        come from the fused kernels, the distribution object is torch's."""
        from . import ops
        from torch import distributions as td
        mu, std = ops.policy_params(self, states)
        return td.Independent(SquashedGaussian(mu, std), 1)

    def act1(self, state, eval=False, noise=None):
        return self.act(torch.unsqueeze(state, 0), eval, noise)[0]

    def copy_from(self, other):
        self.group.data.copy_(other.group.data)


class UniformPolicy:
    """Warm-up policy (src/policy.py:20-58): a ~ U[low, high) per action dim, drawn on
    the device (or taken from a recorded tape in parity mode)."""

    def __init__(self, env_or_action_space, device=None, noise=None):
        space = getattr(env_or_action_space, 'action_space', env_or_action_space)
        from .torch_util import device as default_device
        self.device = default_device if device is None else device
        self.low = torch.as_tensor(np.asarray(space.low, np.float32), device=self.device)
        self.high = torch.as_tensor(np.asarray(space.high, np.float32), device=self.device)
        self.shape = list(space.shape)
        self.noise = noise

    def act(self, states, eval, noise=None):
        noise = noise or self.noise
        n = len(states)
        u = None if noise is None else noise.rand((n, *self.shape))
        if u is None:
            u = torch.rand(n, *self.shape, device=self.device)
        else:
            u = torch.from_numpy(u).to(self.device)
        return self.low + u * (self.high - self.low)

    def act1(self, state, eval=False, noise=None):
        return self.act(torch.unsqueeze(state, 0), eval, noise)[0]
