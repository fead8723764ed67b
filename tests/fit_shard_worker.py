"""Worker for tests/test_gpu_dp.py::test_member_sharded_fit_two_ranks.

One process per rank (RANK / WORLD_SIZE / MASTER_* in the environment, gloo for
the exchange, both ranks on the one MI355X). Each rank fits ITS members of the
golden 4-member ensemble (distributed.MemberShard) on its slice of the recorded
randint draws, exchanging only the log-var bound gradients per step; after the
fit every rank must hold the single-process reference's parameters for ALL
members, its per-step losses and its elites. Exit code 0 = parity."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def main():
    import numpy as np
    import torch
    import torch.distributed as dist
    env = sys.argv[1]
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    torch.set_num_threads(2)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import drpo_amd
    from drpo_amd.distributed import member_sharding
    from conftest import load_golden
    from test_gpu_ensemble import model_from, fill, check_sd
    d = load_golden(f'ensemble_{env}')
    alg, m = model_from(d, env)
    sh = member_sharding(m)
    assert sh is not None and sh.count == m.ensemble_size // world
    if rank == 1:
        # diverge every parameter, then restore only this rank's own members and the
        # shared bounds: the other members must come back through the post-fit gather
        m.group.data.add_(0.5)
        for k in d.files:
            if not k.startswith('sd/') or k[3:] not in m.group.entries:
                continue
            view, v = m.group.view(k[3:]), torch.from_numpy(np.array(d[k])).to(m.group.data.device)
            if k.endswith('log_var'):
                view.copy_(v)
            else:
                view[sh.z0:sh.z1].copy_(v[sh.z0:sh.z1])
    fill(alg, d)
    tape = drpo_amd.TapeNoise.from_npz(d, 'fit_tape')
    losses = m.fit(alg.replay_buffer, steps=3, noise=tape)
    torch.cuda.synchronize()
    assert tape.done()
    np.testing.assert_allclose(losses, d['out/fit_losses'], rtol=1e-4)
    assert m._elite_inds == list(d['out/elite_inds']), (m._elite_inds, list(d['out/elite_inds']))
    check_sd(m, d, 'fit_sd/')
    dist.barrier()
    dist.destroy_process_group()
    print(f'rank {rank}: member-sharded fit parity ok')


if __name__ == '__main__':
    main()
