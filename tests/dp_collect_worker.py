"""Worker for tests/test_gpu_dp.py::test_dp_collection_replicas_agree.

Production data parallelism through the real-env driver: every rank builds the same
SMBPO (seeded alike, identically seeded point-robot envs) and runs setup()
(uniform-policy collection to buffer_min + the initial fit) and a few steps of the
step generator (actor actions with the safety shield, model fits every 4 steps,
rollout_and_update). The collection draws come from DeviceNoise.collection(), which
is the same on every rank, so every replica must hold the same real replay buffer,
the same state normalizer, the same reward bounds and bit-identical parameters,
while the imagined rollouts (per-rank Philox) differ. ``mode`` picks the model-fit
data parallelism: 'batch' (gradient all-reduce) or 'members' (ensemble shard).
Exit 0 = ok."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def main():
    import numpy as np
    import torch
    import torch.distributed as dist
    mode = sys.argv[1]
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    torch.set_num_threads(2)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import drpo_amd
    from pr_env import PointRobot, TorchEnv
    dev = torch.device('cuda', 0)
    # a driver that seeds torch per rank (seed + rank): DeviceNoise(seed=None) must
    # still share rank 0's base seed
    drpo_amd.set_seed(11 + rank)
    rs = np.random.RandomState(5)
    resets = [np.array([rs.uniform(-2, 0), rs.uniform(-2, 0), 1.0, rs.uniform(0.5, 1.2)]) for _ in range(64)]
    factory = lambda id=None: TorchEnv(PointRobot(id=id, resets=list(resets)), dev)  # noqa: E731
    cfg = drpo_amd.SMBPO.Config()
    hid = 64
    cfg.update({'horizon': 3, 'rollout_batch_size': 64, 'buffer_max': 4096, 'buffer_min': 120,
                'steps_per_epoch': 6, 'model_update_period': 4, 'model_initial_steps': 3, 'model_steps': 2,
                'solver_updates_per_step': 2, 'safe_shield': True, 'safe_shield_threshold': -0.1,
                'model_cfg': {'ensemble_size': 4, 'num_elites': 3, 'hidden_dim': 40, 'batch_size': 32,
                              'holdout_size': 32, 'dp_mode': mode},
                'sac_cfg': {'batch_size': 64, 'hidden_dim': hid, 'critic_cfg': {'hidden_dim': hid},
                            'constraint_critic_cfg': {'hidden_dim': hid},
                            'mlp_multiplier_cfg': {'hidden_dim': hid}, 'target_entropy': -2.0},
                'reward_scale': 2.0, 'alive_bonus': 1.0})
    alg = drpo_amd.SMBPO(cfg, factory, None, 1, device=dev)
    assert alg.noise.base_seed == 11, alg.noise.base_seed
    from drpo_amd.distributed import sync_parameters
    sync_parameters(alg)
    alg.setup()
    for _ in range(6):
        next(alg.stepper)
    torch.cuda.synchronize()
    sol, m = alg.solver, alg.model_ensemble
    real = torch.cat([alg.replay_buffer.get('states').reshape(-1), alg.replay_buffer.get('actions').reshape(-1)])
    virt = alg.virt_buffer.get('states')[:32].reshape(-1).contiguous()
    norm = torch.cat([m.state_normalizer.mean, m.state_normalizer.std])
    bounds = torch.tensor([sol.r_min, sol.r_max], dtype=torch.float64)
    flat = torch.cat([sol.critic_group.data, sol.actor.group.data, sol.actor_safe.group.data,
                      sol.multiplier_group.data, sol.log_alpha.view(1), m.group.data])

    def gather(t):
        t = t.detach().cpu().contiguous()
        out = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        return out

    checks = {'real buffer': gather(real), 'normalizer': gather(norm), 'reward bounds': gather(bounds),
              'parameters': gather(flat), 'elites': gather(torch.tensor(m._elite_inds))}
    for name, vals in checks.items():
        for r in range(1, world):
            assert torch.equal(vals[0], vals[r]), f'rank {r} {name} differs from rank 0'
    vs = gather(virt)
    assert not torch.equal(vs[0], vs[1]), 'imagined rollouts should be independent shards'
    assert torch.isfinite(flat).all()
    dist.barrier()
    dist.destroy_process_group()
    print(f'rank {rank}: {len(alg.replay_buffer)} real rows, replicas agree ({mode})')


if __name__ == '__main__':
    main()
