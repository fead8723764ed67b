"""Worker for tests/test_gpu_dp.py::test_device_noise_replicas_stay_identical.

Production data parallelism with DeviceNoise: every rank builds the same SMBPO
(same seed) and calls rollout_and_update twice with its own Philox stream (the
device key mixes in the rank) but the shared host choices (elite member, critic
pick). The rollouts must differ across ranks (independent shards) while the
parameters after the mean-all-reduced updates must be bit-identical on every rank
(one well-defined loss per step, src/ssac.py:437-578 under DP). Exit 0 = ok."""
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
    torch.set_num_threads(2)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import bench
    dev = torch.device('cuda', 0)
    alg = bench.make_alg(dev, 512, 5, 7, 3, bench.QUAD_JSON)
    assert alg.noise.rank == rank and alg.noise.base_seed == 3
    rep = bench.synth_replay('quadrotor', 20000, np.random.RandomState(0), dev, alg.env_params)
    alg.replay_buffer.extend(**{k: torch.from_numpy(v).to(dev) for k, v in rep.items()})
    alg.model_ensemble.state_normalizer.fit(alg.replay_buffer.get('states'))
    alg.model_ensemble._elite_inds = [0, 2, 4, 6, 1]
    for _ in range(2):
        alg.rollout_and_update()
    torch.cuda.synchronize()
    s0 = alg.virt_buffer.get('states')[:64].contiguous()
    flat = torch.cat([alg.solver.critic_group.data, alg.solver.actor.group.data, alg.solver.actor_safe.group.data,
                      alg.solver.multiplier_group.data, alg.solver.log_alpha.view(1)]).contiguous()
    gathered = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    states = [torch.empty_like(s0) for _ in range(world)]
    dist.all_gather(states, s0)
    for r in range(1, world):
        assert torch.equal(gathered[0], gathered[r]), f'rank {r} parameters differ from rank 0'
        assert not torch.equal(states[0], states[r]), f'rank {r} rolled out the same rows as rank 0'
    assert torch.isfinite(flat).all()
    dist.barrier()
    dist.destroy_process_group()
    print(f'rank {rank}: replicas identical, shards independent')


if __name__ == '__main__':
    main()
