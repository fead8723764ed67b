"""Probabilistic dynamics ensemble (src/dynamics.py:55-253) on flat HBM parameters.

Residual Gaussian MLP ensemble: trunk [S+A -> H -> H] (swish, swish output),
diff head and log-var head [H -> H -> S+1] (swish hidden), learned soft log-var
bounds. Weights are [E, out, in] (BatchedLinear layout). Forward passes run the
fused HIP MLP kernels (ops.py); the member forward used by rollouts is fused into
the rollout kernel (csrc/rollout.hip)."""
import torch
import torch.nn as nn

from .config import BaseConfig, Configurable
from .params import FlatGroup, MLPSpec, layer_views
from .torch_util import Module, device as default_device


class Normalizer(Module):
    """src/normalization.py:6-27."""

    def __init__(self, dim, epsilon=1e-6, device=default_device):
        super().__init__()
        self.dim = dim
        self.epsilon = epsilon
        self.register_buffer('mean', torch.zeros(dim, device=device))
        self.register_buffer('std', torch.zeros(dim, device=device))

    def fit(self, X):
        from . import ops
        assert torch.is_tensor(X) and X.dim() == 2 and X.shape[1] == self.dim
        ops.normalizer_fit(X, self.mean, self.std)

    def forward(self, x):
        from . import ops
        return ops.normalize(x, self.mean, self.std, self.epsilon)


class BatchedGaussianEnsemble(Configurable, Module):
    class Config(BaseConfig):
        ensemble_size = 7
        num_elites = 5
        hidden_dim = 200
        trunk_layers = 2
        head_hidden_layers = 1
        activation = 'swish'
        init_min_log_var = -10.0
        init_max_log_var = 1.0
        log_var_bound_weight = 0.01
        batch_size = 256
        learning_rate = 1e-3
        holdout_size = 256
        # multi-GPU fit: 'auto' shards members over ranks when E >= world size
        # (distributed.MemberShard), 'batch' all-reduces whole-ensemble gradients
        dp_mode = 'auto'

    def __init__(self, config, state_dim, action_dim, device=default_device, optimizer_factory=None):
        Configurable.__init__(self, config)
        Module.__init__(self)
        assert self.activation == 'swish', 'fused kernels implement the reference swish ensemble'
        self.state_dim, self.action_dim = state_dim, action_dim
        E, H = self.ensemble_size, self.hidden_dim
        in_dim, out_dim = state_dim + action_dim, state_dim + 1
        self.trunk_spec = MLPSpec([in_dim] + [H] * self.trunk_layers, 'swish', 'swish', ensemble=E)
        head = [H] * (self.head_hidden_layers + 1) + [out_dim]
        self.diff_spec = MLPSpec(head, 'swish', ensemble=E)
        self.logvar_spec = MLPSpec(head, 'swish', ensemble=E)

        g = FlatGroup('model')
        self.trunk_spec.register(g, 'trunk.')
        self.diff_spec.register(g, 'diff_head.')
        self.logvar_spec.register(g, 'log_var_head.')
        g.add('min_log_var', (out_dim,))
        g.add('max_log_var', (out_dim,))
        g.allocate('cpu')
        g.view('min_log_var').fill_(self.init_min_log_var)
        g.view('max_log_var').fill_(self.init_max_log_var)
        # reference order: trunk, diff_head, log_var_head (each: constructions then xavier)
        self.trunk_spec.reference_init(g, 'trunk.')
        self.diff_spec.reference_init(g, 'diff_head.')
        self.logvar_spec.reference_init(g, 'log_var_head.')
        g.data, g.grad = g.data.to(device), g.grad.to(device)
        from .params import spec_pack_layers
        g.enable_packing(spec_pack_layers(self.trunk_spec, 'trunk.') + spec_pack_layers(self.diff_spec, 'diff_head.') +
                         spec_pack_layers(self.logvar_spec, 'log_var_head.'))
        self.group = g

        self.min_log_var = nn.Parameter(g.view('min_log_var'), requires_grad=False)
        self.max_log_var = nn.Parameter(g.view('max_log_var'), requires_grad=False)
        self.min_log_var.grad = g.view('min_log_var', g.grad)
        self.max_log_var.grad = g.view('max_log_var', g.grad)
        self.state_normalizer = Normalizer(state_dim, device=device)
        self.trunk = self.trunk_spec.build(g, 'trunk.')
        self.diff_head = self.diff_spec.build(g, 'diff_head.')
        self.log_var_head = self.logvar_spec.build(g, 'log_var_head.')

        from .optim import Adam
        self.optimizer = Adam(g, lr=self.learning_rate, weight_decay=1e-4)
        self._init_elites()

    def _init_elites(self):
        # CPU generator draw, as src/dynamics.py:105-106
        self.elite_inds = torch.randint(high=self.ensemble_size, size=(self.num_elites,)).tolist()

    @property
    def total_batch_size(self):
        return self.ensemble_size * self.batch_size

    # weight views --------------------------------------------------------
    def views(self, buf=None):
        g = self.group
        return (layer_views(g, 'trunk.', self.trunk_spec, buf), layer_views(g, 'diff_head.', self.diff_spec, buf),
                layer_views(g, 'log_var_head.', self.logvar_spec, buf))

    # API (compute in ensemble_engine.py) ------------------------------------
    @property
    def engine(self):
        eng = self.__dict__.get('_engine')
        if eng is None:
            from .ensemble_engine import EnsembleEngine
            eng = EnsembleEngine(self)
            self.__dict__['_engine'] = eng
        return eng

    def _forward1(self, states, actions, index):
        return self.engine.forward1(states, actions, index)

    def _forward_all(self, states, actions):
        return self.engine.forward_all(states, actions)

    def _rebatch(self, x):
        n = len(x)
        assert n % self.ensemble_size == 0, f'{n} not divisible by {self.ensemble_size}'
        return x.reshape(self.ensemble_size, n // self.ensemble_size, *x.shape[1:])

    def sample(self, states, actions, noise=None):
        import random
        index = self._elite_inds[random.choice(range(len(self._elite_inds))) if noise is None
                                 else noise.choice(len(self._elite_inds))]
        return self.engine.sample(states, actions, index, noise)

    def means(self, states, actions):
        # states.repeat(E, 1, 1) of the reference == member stride 0 (no copy)
        means, _ = self._forward_all(states.unsqueeze(0), actions.unsqueeze(0))
        return means[:, :, :-1], means[:, :, -1]

    def mean(self, states, actions):
        s, r = self.means(states, actions)
        return s.mean(dim=0), r.mean(dim=0)

    def elite_samples(self, states, actions, noise=None):
        return self.engine.elite_samples(states, actions, list(self._elite_inds), noise)

    def compute_loss(self, states, actions, targets):
        from .ensemble_engine import EnsembleLoss
        anchor = self.__dict__.get('_anchor')
        if anchor is None:
            anchor = self.__dict__['_anchor'] = torch.zeros((), requires_grad=True)
        if torch.is_grad_enabled():
            return EnsembleLoss.apply(anchor, self.engine, states, actions, targets)
        return self.engine.compute_loss_value(states, actions, targets)

    def _mse_loss(self, states, actions, targets, enable_grad=True):
        """Per-member NLL [E] (values only; gradients flow through compute_loss)."""
        e = self.engine
        s, a, t = e._prep(states, actions, targets)
        E, b, S = s.shape
        nets, _, _ = e._forward(s, a, b, E, b * S, b * self.action_dim, tag='mse')
        mse, _, _ = e._loss(nets, s, b * S, t, b * (S + 1), b, E, False, tag='mse')
        return mse.clone()

    def fit(self, buffer, steps=None, epochs=None, progress_bar=False, noise=None, **kwargs):
        if steps is not None:
            assert epochs is None, 'Cannot pass both steps and epochs'
            return self.engine.fit(buffer, steps, noise)
        if epochs is not None:
            return self.engine.fit_epochs(buffer, epochs, **kwargs)
        raise ValueError('Must pass steps or epochs')
