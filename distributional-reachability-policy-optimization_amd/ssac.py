"""Safe SAC solver with the distributional reachability certificate (src/ssac.py:17-600).

Networks live in flat HBM parameter groups (params.py):
  critic group   = twin Q critics + constraint critic (one optimizer in the reference,
                   two separate grad-norm clips), with an identically laid-out target group
  actor / actor_safe / multiplier groups, plus the scalar log_alpha.
The update methods run the HIP kernels orchestrated in sac_step.py; the module
tree (and therefore state_dict keys/shapes) matches the reference exactly.
"""
import math

import torch
import torch.nn as nn

from .config import BaseConfig, Configurable, Optional
from .params import FlatGroup, MLPSpec
from .policy import SquashedGaussianPolicy
from .torch_util import Module, device as default_device


class CriticEnsemble(Configurable, Module):
    class Config(BaseConfig):
        n_critics = 2
        hidden_layers = 2
        hidden_dim = 256

    def __init__(self, config, state_dim, action_dim, group=None, prefix='critic.'):
        Configurable.__init__(self, config)
        Module.__init__(self)
        self.spec = MLPSpec([state_dim + action_dim, *([self.hidden_dim] * self.hidden_layers), 1], 'relu',
                            squeeze=True)
        self.group, self.prefix = group, prefix

    def register(self, g):
        for i in range(self.n_critics):
            self.spec.register(g, f'{self.prefix}qs.{i}.')

    def reference_init(self, g):
        for i in range(self.n_critics):
            self.spec.reference_init(g, f'{self.prefix}qs.{i}.')

    def build(self, g, prefix=None):
        prefix = self.prefix if prefix is None else prefix
        self.group, self.prefix = g, prefix
        self.qs = nn.ModuleList([self.spec.build(g, f'{prefix}qs.{i}.') for i in range(self.n_critics)])

    def all(self, state, action):
        from . import ops
        return ops.critic_all(self, state, action)

    def min(self, state, action):
        return torch.min(*self.all(state, action))

    def mean(self, state, action):
        qs = self.all(state, action)
        return sum(qs) / len(qs)

    def random_choice(self, state, action, noise=None):
        import random
        from . import ops
        i = random.choice(range(self.n_critics)) if noise is None else noise.choice(self.n_critics)
        return ops.critic_all(self, state, action, which=[i])[0]


class ConstraintCritic(Configurable, Module):
    class Config(BaseConfig):
        trunk_layers = 2
        head_layers = 1
        hidden_dim = 256
        log_std_min = -4.
        log_std_max = 4.
        std_ratio = 2.

    def __init__(self, config, state_dim, action_dim, output_dim, output_activation=None, group=None,
                 prefix='constraint_critic.'):
        Configurable.__init__(self, config)
        Module.__init__(self)
        H = self.hidden_dim
        self.output_dim = output_dim
        self.trunk_spec = MLPSpec([state_dim + action_dim] + [H] * self.trunk_layers, 'relu', 'relu')
        head = [H] * (self.head_layers + 1) + [output_dim]
        self.mean_spec = MLPSpec(head, 'relu', squeeze=True)
        self.logstd_spec = MLPSpec(head, 'relu', squeeze=True)
        self.group, self.prefix = group, prefix

    def register(self, g):
        self.trunk_spec.register(g, self.prefix + 'trunk.')
        self.mean_spec.register(g, self.prefix + 'mean_head.')
        self.logstd_spec.register(g, self.prefix + 'log_std_head.')

    def reference_init(self, g):
        self.trunk_spec.reference_init(g, self.prefix + 'trunk.')
        self.mean_spec.reference_init(g, self.prefix + 'mean_head.')
        self.logstd_spec.reference_init(g, self.prefix + 'log_std_head.')

    def build(self, g, prefix=None):
        prefix = self.prefix if prefix is None else prefix
        self.group, self.prefix = g, prefix
        self.trunk = self.trunk_spec.build(g, prefix + 'trunk.')
        self.mean_head = self.mean_spec.build(g, prefix + 'mean_head.')
        self.log_std_head = self.logstd_spec.build(g, prefix + 'log_std_head.')

    def forward(self, state, action, uncertainty=False, sample=False, noise=None):
        from . import ops
        return ops.constraint_critic_forward(self, state, action, uncertainty, sample, noise)


class MLPMultiplier(Configurable, Module):
    class Config(BaseConfig):
        hidden_layers = 2
        hidden_dim = 256
        upper_bound = 50.

    def __init__(self, config, state_dim, group=None, prefix='multiplier.'):
        Configurable.__init__(self, config)
        Module.__init__(self)
        self.spec = MLPSpec([state_dim + 1, *([self.hidden_dim] * self.hidden_layers), 1], 'tanh', 'identity',
                            squeeze=True)
        self.group, self.prefix = group, prefix

    def forward(self, state, Qc):
        from . import ops
        return ops.multiplier_forward(self, state, Qc)


class SSAC(Module):
    class Config(BaseConfig):
        discount = 0.99
        init_alpha = 1.0
        autotune_alpha = True
        target_entropy = Optional(float)
        use_log_alpha_loss = False
        deterministic_backup = False
        critic_update_multiplier = 1
        actor_lr = 8e-5
        actor_lr_end = 4e-5
        critic_lr = 3e-4
        critic_lr_end = 8e-5
        multiplier_lr = 3e-4
        multiplier_lr_end = 1e-5
        critic_cfg = CriticEnsemble.Config()
        constraint_critic_cfg = ConstraintCritic.Config()
        mlp_multiplier_cfg = MLPMultiplier.Config()
        tau = 0.005
        actor_update_interval = 2
        batch_size = 256
        hidden_dim = 256
        hidden_layers = 2
        update_violation_cost = False
        grad_norm = 5.
        constraint_threshold = 0.
        constrained_fcn = 'reachability'
        mlp_multiplier = True
        penalty_lb = -1.0
        penalty_ub = 100.
        fixed_multiplier = 15.0
        multiplier_update_interval = 5
        lam_epsilon = 1.0
        qc_under_uncertainty = True
        qc_td_bound = 5.
        distributional_qc = True

    def __init__(self, config, state_dim, action_dim, con_dim, horizon, epochs, steps_per_epoch,
                 solver_updates_per_step, constraint_scale, env_factory, model_ensemble,
                 optimizer_factory=None, device=default_device):
        assert type(config) is SSAC.Config
        Module.__init__(self)
        import copy
        self.config = copy.deepcopy(config)
        for k, v in vars(self.config).items():
            setattr(self, k, v)
        if isinstance(self.target_entropy, Optional):
            self.target_entropy = None
        assert self.constrained_fcn in ('reachability', 'cost'), self.constrained_fcn
        if self.constrained_fcn == 'cost':
            # the reference's cost branch runs only where it does not crash: compute_cons_target
            # returns one target, which the distributional loss unpacks as two (src/ssac.py:430-431),
            # and _get_qc of the single-output critic asserts for con_dim > 1 behind the MLP
            # multiplier (src/ssac.py:476,548)
            assert not self.distributional_qc, "constrained_fcn='cost' needs distributional_qc=False"
            assert con_dim == 1 or not self.mlp_multiplier, \
                "constrained_fcn='cost' with con_dim > 1 needs mlp_multiplier=False"
        self.state_dim, self.action_dim, self.con_dim = state_dim, action_dim, con_dim
        self.horizon = horizon
        self.violation_cost = 0.0
        self.updates_per_training = epochs * steps_per_epoch * solver_updates_per_step
        self.lam_updates_num = int(self.updates_per_training / self.multiplier_update_interval)
        self.actor_updates_num = int(self.updates_per_training / self.actor_update_interval)
        self.env = env_factory()
        self.constraint_scale = constraint_scale
        self.model_ensemble = model_ensemble

        # ---- networks (reference construction / RNG order, src/ssac.py:184-253) ----
        self.actor = SquashedGaussianPolicy.create(state_dim, action_dim, self.hidden_dim, self.hidden_layers,
                                                   'actor', device)
        self.actor_safe = SquashedGaussianPolicy.create(state_dim, action_dim, self.hidden_dim,
                                                        self.hidden_layers, 'actor_safe', device, init=False)
        self.actor_safe.copy_from(self.actor)

        cg = FlatGroup('critic')
        critic = CriticEnsemble(self.critic_cfg, state_dim, action_dim, prefix='critic.')
        # certificate width: one output per constraint, or one cost value (src/ssac.py:191-195;
        # the reference's softplus output_activation is accepted and ignored there, :55-62)
        cc_out = con_dim if self.constrained_fcn == 'reachability' else 1
        cc = ConstraintCritic(self.constraint_critic_cfg, state_dim, action_dim, cc_out,
                              prefix='constraint_critic.')
        critic.register(cg)
        cc.register(cg)
        cg.allocate('cpu')
        critic.reference_init(cg)
        cc.reference_init(cg)
        cg.data, cg.grad = cg.data.to(device), cg.grad.to(device)
        tg = FlatGroup('critic_target')
        tg.entries, tg.order, tg.size = dict(cg.entries), list(cg.order), cg.size
        tg.data, tg.grad = cg.data.clone(), None
        from .params import spec_pack_layers
        crit_layers = [x for i in range(critic.n_critics) for x in spec_pack_layers(critic.spec, f'critic.qs.{i}.')]
        crit_layers += (spec_pack_layers(cc.trunk_spec, 'constraint_critic.trunk.') +
                        spec_pack_layers(cc.mean_spec, 'constraint_critic.mean_head.') +
                        spec_pack_layers(cc.logstd_spec, 'constraint_critic.log_std_head.'))
        cg.enable_packing(crit_layers)
        tg.enable_packing(crit_layers, transposed=False)
        critic.build(cg, 'critic.')
        cc.build(cg, 'constraint_critic.')
        critic_t = CriticEnsemble(self.critic_cfg, state_dim, action_dim, prefix='critic.')
        critic_t.build(tg, 'critic.')
        cc_t = ConstraintCritic(self.constraint_critic_cfg, state_dim, action_dim, cc_out,
                                prefix='constraint_critic.')
        cc_t.build(tg, 'constraint_critic.')
        self.critic, self.critic_target = critic, critic_t
        self.constraint_critic, self.constraint_critic_target = cc, cc_t
        self.critic_group, self.critic_target_group = cg, tg

        self.log_alpha = torch.tensor(math.log(self.init_alpha), device=device)
        if self.target_entropy is None:
            self.target_entropy = -action_dim

        # multiplier (src/ssac.py:232-252): the state-dependent MLP, or one scalar
        # parameter (init 10, lambda = softplus) in its own one-element flat group
        mg = FlatGroup('multiplier')
        if self.mlp_multiplier:
            mult = MLPMultiplier(self.mlp_multiplier_cfg, state_dim, prefix='lam.')
            mult.spec.register(mg, 'lam.')
            mg.allocate('cpu')
            mult.spec.reference_init(mg, 'lam.')
            mg.data, mg.grad = mg.data.to(device), mg.grad.to(device)
            mg.enable_packing(spec_pack_layers(mult.spec, 'lam.'))
            mult.lam = mult.spec.build(mg, 'lam.')
            mult.group = mg
            self.multiplier = mult
        else:
            mg.add('multiplier', ())
            mg.allocate(device)
            mg.data[0] = 10.
            self.multiplier = torch.nn.Parameter(mg.view('multiplier'), requires_grad=False)
            self.multiplier.grad = mg.view('multiplier', mg.grad)
        self.multiplier_group = mg

        from .optim import Adam, CosineAnnealingLR
        T = self.updates_per_training
        self.critic_optimizer = Adam(cg, lr=self.critic_lr, weight_decay=1e-4)
        self.critic_lr_scheduler = CosineAnnealingLR(self.critic_optimizer, T, self.critic_lr_end)
        self.actor_optimizer = Adam(self.actor.group, lr=self.actor_lr, weight_decay=1e-4)
        self.actor_lr_scheduler = CosineAnnealingLR(self.actor_optimizer, self.actor_updates_num, self.actor_lr_end)
        self.actor_safe_optimizer = Adam(self.actor_safe.group, lr=self.actor_lr, weight_decay=1e-4)
        self.actor_safe_lr_scheduler = CosineAnnealingLR(self.actor_safe_optimizer, self.actor_updates_num,
                                                         self.actor_lr_end)
        self.alpha_optimizer = Adam(None, lr=self.actor_lr, weight_decay=0.0)   # stepped only if autotune_alpha
        if self.mlp_multiplier:
            self.multiplier_optimizer = Adam(mg, lr=self.multiplier_lr, weight_decay=1e-4)
            self.multiplier_lr_scheduler = CosineAnnealingLR(self.multiplier_optimizer, self.lam_updates_num,
                                                             self.multiplier_lr_end)
        else:   # plain Adam at a fixed lr (no weight decay, no schedule)
            self.multiplier_optimizer = Adam(mg, lr=self.multiplier_lr, weight_decay=0.0)
            self.multiplier_lr_scheduler = None
        self.register_buffer('total_updates', torch.zeros([], device=device))
        self._engine = None

    # ------------------------------------------------------------------
    def act(self, states, eval, noise=None):
        return self.actor.act(states, eval, noise)

    @property
    def alpha(self):
        return self.log_alpha.exp()

    @property
    def lam(self):
        """softplus(multiplier) of the scalar-multiplier configuration (src/ssac.py:261-265)."""
        assert not self.mlp_multiplier
        assert self.multiplier.shape == ()
        return torch.nn.functional.softplus(self.multiplier.detach())

    @property
    def violation_value(self):
        return -self.violation_cost / (1. - self.discount)

    def update_r_bounds(self, r_min, r_max):
        self.r_min, self.r_max = r_min, r_max
        if self.update_violation_cost:
            self.violation_cost = (r_max - r_min) / self.discount ** self.horizon - r_max

    def _get_qc(self, qc_con_dim):
        if self.con_dim > 1:
            assert qc_con_dim.size(-1) == self.con_dim
            return torch.max(qc_con_dim, dim=-1)[0]
        return qc_con_dim

    @property
    def engine(self):
        if self._engine is None:
            from .sac_step import SACEngine
            self._engine = SACEngine(self)
        return self._engine

    def update_critic(self, *critic_loss_args, noise=None):
        return self.engine.update_critic(*critic_loss_args, noise=noise)

    def update_actor_and_alpha(self, obs, noise=None):
        return self.engine.update_actor_and_alpha(obs, noise=noise)

    def update_multiplier(self, obs, noise=None):
        return self.engine.update_multiplier(obs, noise=noise)

    def update(self, replay_buffer):
        for _ in range(self.critic_update_multiplier):
            samples = replay_buffer.sample(self.batch_size)
            self.update_critic(*samples)
        self.update_actor_and_alpha(samples[0])
        self.total_updates += 1
