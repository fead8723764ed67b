"""Worker for the data-parallel parity tests (tests/test_gpu_dp.py, tests/test_distributed.py).

Run as one process per rank (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the
environment). Each rank takes its row shard of a golden SSAC fixture batch and
of every batch-shaped recorded draw, runs update_critic -> update_actor_and_alpha
-> update_multiplier with gradients mean-all-reduced across ranks, and checks
the parameters against the single-process reference result after every update
(the losses are batch means, so the mean of equal-shard gradients is the
full-batch gradient). Exit code 0 = parity."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def shard_tape(entries, B, rank, world):
    out = []
    for kind, v in entries:
        if getattr(v, 'ndim', 0) >= 1 and v.shape[0] == B:
            n = B // world
            v = v[rank * n:(rank + 1) * n]
        out.append((kind, v))
    return out


def main():
    import numpy as np
    import torch
    import torch.distributed as dist
    tag, backend = sys.argv[1], sys.argv[2]
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    torch.set_num_threads(2)
    dist.init_process_group(backend, rank=rank, world_size=world)
    import drpo_amd
    from drpo_amd.distributed import sync_parameters
    from conftest import load_golden
    from gpu_helpers import DEV, small_smbpo
    from test_gpu_sac import solver_sd, check_params
    d = load_golden(f'ssac_{tag}')
    alg = small_smbpo(d, str(d['meta/env']))
    sol = alg.solver
    sd0 = solver_sd(d, 'sd0/')
    sol.log_alpha.fill_(float(sd0.pop('log_alpha')))
    sol.load_state_dict(sd0, strict=False)
    if 'model/elite_inds' in d.files:
        alg.model_ensemble._elite_inds = list(d['model/elite_inds'])
    if rank == 1:                       # diverge, then resync from rank 0
        sol.critic_group.data.add_(1.0)
    sync_parameters(alg)
    B = d['in/s'].shape[0]
    n = B // world
    batch = [torch.from_numpy(d['in/' + k][rank * n:(rank + 1) * n]).to(DEV) for k in ['s', 'a', 's2', 'r', 'd', 'v',
                                                                                       'h']]

    def tape(name):
        t = drpo_amd.TapeNoise.from_npz(d, name)
        return drpo_amd.TapeNoise(shard_tape(t.entries, B, rank, world))

    from drpo_amd.distributed import CommLog

    def one_bucket(phase, c0):   # each update exchanges ONE all-reduce bucket
        n = CommLog.calls - c0
        assert n == 1, f'rank {rank}: {phase} issued {n} collectives'

    c0 = CommLog.calls
    sol.update_critic(*batch, noise=tape('critic_tape'))
    torch.cuda.synchronize()
    one_bucket('update_critic', c0)
    check_params(sol, solver_sd(d, 'sd1/'), f'rank {rank} after update_critic')
    c0 = CommLog.calls
    sol.update_actor_and_alpha(batch[0], noise=tape('actor_tape'))
    torch.cuda.synchronize()
    one_bucket('update_actor_and_alpha', c0)
    ref2 = solver_sd(d, 'sd2/')
    np.testing.assert_allclose(sol.log_alpha.item(), float(ref2['log_alpha']), rtol=1e-5, atol=1e-6)
    check_params(sol, ref2, f'rank {rank} after update_actor_and_alpha')
    c0 = CommLog.calls
    sol.update_multiplier(batch[0], noise=tape('mult_tape'))
    torch.cuda.synchronize()
    one_bucket('update_multiplier', c0)
    check_params(sol, solver_sd(d, 'sd3/'), f'rank {rank} after update_multiplier')
    dist.barrier()
    dist.destroy_process_group()
    print(f'rank {rank}: data-parallel parity ok')


if __name__ == '__main__':
    main()
