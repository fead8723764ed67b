"""CPU-only checks of the host side: reference-order initialisation (bit-exact vs
the reference's sha256 per state_dict tensor), state_dict layout, configs."""
import hashlib

import numpy as np
import pytest
import torch

import drpo_amd
from conftest import load_golden
from fake_envs import ENVS


def make_smbpo(env, device='cpu', seed=0, epochs=100, **upd):
    cfg = drpo_amd.SMBPO.Config()
    cfg.update({'sac_cfg': {'qc_under_uncertainty': True, 'distributional_qc': True}})
    if upd:
        cfg.update(upd)
    drpo_amd.set_seed(seed)
    return drpo_amd.SMBPO(cfg, lambda id=None: ENVS[env](), None, epochs, device=torch.device(device))


def test_reference_init_bit_exact():
    d = load_golden('init_hashes_quadrotor')
    alg = make_smbpo('quadrotor')
    sd = alg.state_dict()
    ref_keys = [k[len('hash/'):] for k in d.files if k.startswith('hash/')]
    assert sorted(sd.keys()) == sorted(ref_keys)
    for k in ref_keys:
        arr = np.ascontiguousarray(sd[k].detach().cpu().numpy())
        assert tuple(arr.shape) == tuple(d['shape/' + k]), k
        assert str(arr.dtype) == str(d['dtype/' + k]), k
        assert hashlib.sha256(arr.tobytes()).hexdigest() == str(d['hash/' + k]), k
    assert alg.model_ensemble.elite_inds == list(d['elite_inds'])


def test_state_dict_order_and_duplicates():
    alg = make_smbpo('point-robot')
    keys = list(alg.state_dict().keys())
    assert keys[:4] == ['episodes_sampled', 'steps_sampled', 'n_violations', 'epochs_completed']
    assert 'solver.model_ensemble.trunk.0.weight' in keys          # duplicated sub-module, like the reference
    assert 'solver.log_alpha' not in keys                            # not saved by the reference either
    assert alg.state_dict()['model_ensemble.trunk.0.weight'].shape == (7, 200, 13)


def test_state_dict_round_trip_aliases_flat_storage():
    a = make_smbpo('point-robot', seed=1)
    b = make_smbpo('point-robot', seed=2)
    b.load_state_dict(a.state_dict())
    assert torch.equal(a.solver.critic_group.data, b.solver.critic_group.data)
    assert torch.equal(a.model_ensemble.group.data, b.model_ensemble.group.data)
    assert torch.equal(a.solver.actor.group.data, b.solver.actor.group.data)


def test_config_json_semantics():
    cfg = drpo_amd.SMBPO.Config()
    cfg.update({'sac_cfg': {'target_entropy': -2.0, 'constraint_critic_cfg': {'std_ratio': 2.0}},
                'buffer_max': 360000})
    assert cfg.sac_cfg.target_entropy == -2.0 and cfg.buffer_max == 360000
    assert drpo_amd.SMBPO.Config().buffer_max == 10 ** 6       # class default untouched
    with pytest.raises(AssertionError):
        cfg.update({'horizon': 1.5})
    with pytest.raises(AssertionError):
        cfg.update({'no_such_key': 1})
    cfg.nested_set(['sac_cfg', 'qc_td_bound'], 3.0)
    assert cfg.sac_cfg.qc_td_bound == 3.0


def test_buffer_circular_host_semantics():
    buf = drpo_amd.ConstraintSafetySampleBuffer(3, 2, 5, con_dim=2, device=torch.device('cpu'))
    rows = lambda n, o: dict(states=torch.arange(n * 3).view(n, 3).float() + o, actions=torch.zeros(n, 2),
                             next_states=torch.zeros(n, 3), rewards=torch.arange(n).float() + o,
                             dones=torch.zeros(n, dtype=torch.bool), violations=torch.zeros(n, dtype=torch.bool),
                             constraint_values=torch.zeros(n, 2))
    buf.extend(**rows(3, 0))
    buf.extend(**rows(4, 100))
    assert len(buf) == 5 and buf.pointer == 7
    r = buf.get('rewards')
    assert r.tolist() == [100., 101., 102., 103., 2.][-5:] or r.tolist() == [2., 100., 101., 102., 103.]
    assert r.tolist() == [2., 100., 101., 102., 103.]


def test_actor_exchange_arena_rehomes_parameter_grads():
    """The actor update's single data-parallel bucket: the actor's and
    the safe actor's flat gradients moved into adjacent slices of one arena keep their
    values, and every nn.Parameter's .grad follows into the arena."""
    alg = make_smbpo('quadrotor')
    sol = alg.solver
    ga, gs = sol.actor.group, sol.actor_safe.group
    ga.grad.normal_()
    gs.grad.normal_()
    va, vs = ga.grad.clone(), gs.grad.clone()
    arena = torch.zeros(ga.size + gs.size + 64)
    ga.move_grad(arena[:ga.size], sol.actor)
    gs.move_grad(arena[ga.size:ga.size + gs.size], sol.actor_safe)
    assert torch.equal(arena[:ga.size], va) and torch.equal(arena[ga.size:ga.size + gs.size], vs)
    base, end = arena.data_ptr(), arena.data_ptr() + 4 * arena.numel()
    for mod in (sol.actor, sol.actor_safe):
        for name, p in mod.named_parameters():
            assert p.grad is not None and base <= p.grad.data_ptr() < end, name
    w = sol.actor.net[0].weight
    w.grad.add_(1.0)                      # a write through a parameter's .grad lands in the arena
    assert torch.equal(arena[ga.offset('net.0.weight')], va[ga.offset('net.0.weight')] + 1.0)
