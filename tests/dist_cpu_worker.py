"""Worker for tests/test_distributed.py (gloo, CPU, one process per rank).

Checks the data-parallel plumbing of drpo_amd.distributed without a GPU:
  * GradReducer.mean_ == mean over ranks of each rank's flat buffer;
  * sync_parameters makes every rank's flat groups equal to rank 0's;
  * the DP identity the SAC/ensemble engines rely on: the mean over equal row
    shards of the per-shard gradient of a batch-mean loss equals the full-batch
    gradient (checked on the oracle's critic loss + ensemble NLL)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def main():
    import numpy as np
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    torch.set_num_threads(1)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import drpo_amd
    from drpo_amd.distributed import GradReducer, sync_parameters, world_size, rank as drank
    from conftest import load_golden
    from fake_envs import ENVS
    from oracle import drpo_oracle as O
    assert world_size() == world and drank() == rank
    red = GradReducer()
    assert red.active
    x = torch.arange(10, dtype=torch.float32) * (rank + 1)
    red.mean_(x)
    exp = torch.arange(10, dtype=torch.float32) * sum(r + 1 for r in range(world)) / world
    assert torch.allclose(x, exp), (x, exp)

    # sync_parameters on a CPU-constructed SMBPO (no kernels run)
    cfg = drpo_amd.SMBPO.Config()
    cfg.update({'sac_cfg': {'hidden_dim': 32, 'critic_cfg': {'hidden_dim': 32},
                            'constraint_critic_cfg': {'hidden_dim': 32}, 'mlp_multiplier_cfg': {'hidden_dim': 32}},
                'model_cfg': {'hidden_dim': 24, 'ensemble_size': 3, 'num_elites': 2}, 'buffer_max': 1000})
    torch.manual_seed(100 + rank)      # different init per rank
    alg = drpo_amd.SMBPO(cfg, lambda id=None: ENVS['quadrotor'](), None, 1, device=torch.device('cpu'))
    sync_parameters(alg)
    for t in (alg.solver.critic_group.data, alg.solver.actor.group.data, alg.model_ensemble.group.data):
        ref = t.clone()
        dist.broadcast(ref, 0)
        assert torch.equal(ref, t)

    # DP identity on the oracle: critic (ensemble) loss on half batches, mean of grads
    d = load_golden('ensemble_quadrotor')
    P = {k[3:]: torch.from_numpy(np.array(d[k])) for k in d.files if k.startswith('sd/')}
    P['state_normalizer.mean'] = torch.from_numpy(d['model/norm_mean'])
    P['state_normalizer.std'] = torch.from_numpy(d['model/norm_std'])
    E = int(d['meta/E'])
    s, a = torch.from_numpy(d['replay/states'][:8 * E]), torch.from_numpy(d['replay/actions'][:8 * E])
    t = torch.cat([torch.from_numpy(d['replay/next_states'][:8 * E]),
                   torch.from_numpy(d['replay/rewards'][:8 * E]).unsqueeze(1)], 1)
    keys = O.ens_param_keys(P, '')

    def grads(rows):
        params = {k: P[k].detach().clone().requires_grad_(True) for k in keys}
        Q = dict(P)
        Q.update(params)
        # per-member batch shards: member z takes rows [z*b, (z+1)*b); shard each member's rows
        b = len(s) // E
        idx = torch.cat([torch.arange(z * b, (z + 1) * b)[rows] for z in range(E)])
        loss = O.ens_compute_loss(Q, '', s[idx], a[idx], t[idx], E)
        return torch.autograd.grad(loss, [params[k] for k in keys])

    b = len(s) // E
    full = grads(slice(0, b))
    half = b // world
    mine = grads(slice(rank * half, (rank + 1) * half))
    flat = torch.cat([g.reshape(-1) for g in mine])
    red.mean_(flat)
    # the log-var bound term's gradient (+-0.01) is per-rank constant, so it averages to itself
    ref = torch.cat([g.reshape(-1) for g in full])
    assert torch.allclose(flat, ref, rtol=1e-4, atol=1e-6), float((flat - ref).abs().max())

    # member-sharded fit (distributed.MemberShard): each rank differentiates only its
    # members' NLL terms (+ the log-var bound term on rank 0); member gradients are
    # the full-ensemble gradient's slices, the summed bound gradients its bound part
    from drpo_amd.distributed import MemberShard
    sh = MemberShard(E)
    assert sh.ranges[-1][1] == E and sum(b_ - a_ for a_, b_ in sh.ranges) == E
    Pm = {k: (v[sh.z0:sh.z1] if k in keys and k not in ('min_log_var', 'max_log_var') else v) for k, v in P.items()}
    params = {k: Pm[k].detach().clone().requires_grad_(True) for k in keys}
    Q = dict(Pm)
    Q.update(params)
    rows = torch.cat([torch.arange(z * b, (z + 1) * b) for z in range(sh.z0, sh.z1)])
    loss = O.ens_compute_loss(Q, '', s[rows], a[rows], t[rows], sh.count) if sh.count else torch.zeros(())
    if rank != 0:     # the oracle adds the bound term on every call; only rank 0 keeps it
        loss = loss - 0.01 * (Q['max_log_var'].sum() - Q['min_log_var'].sum())
    g = dict(zip(keys, torch.autograd.grad(loss, [params[k] for k in keys], allow_unused=True)))
    for k, gf in zip(keys, full):
        if k in ('min_log_var', 'max_log_var'):
            gb = g[k].clone()
            sh.sum_(gb)
            assert torch.allclose(gb, gf, rtol=1e-4, atol=1e-6), (k, float((gb - gf).abs().max()))
        else:
            assert torch.allclose(g[k], gf[sh.z0:sh.z1], rtol=1e-4, atol=1e-6), k
    # all-gather of member slices (uneven and even member counts) and holdout merge
    for EE in (7, 8):
        shx = MemberShard(EE)
        w = torch.full((EE, 3, 2), -1.0)
        w[shx.z0:shx.z1] = torch.arange(shx.z0, shx.z1, dtype=torch.float32).view(-1, 1, 1)
        shx.gather_members_(w)
        assert torch.equal(w, torch.arange(EE, dtype=torch.float32).view(-1, 1, 1).expand(EE, 3, 2))
        mse = shx.merge_members(torch.arange(shx.z0, shx.z1, dtype=torch.float32) * 10, torch.zeros(EE))
        assert torch.equal(mse, torch.arange(EE, dtype=torch.float32) * 10)
    dist.barrier()
    dist.destroy_process_group()
    print(f'rank {rank} ok')


if __name__ == '__main__':
    main()
