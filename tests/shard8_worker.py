"""Worker for tests/test_gpu_dp.py::test_member_sharded_fit_e8_four_ranks (config 4's
split: E=8 members over 4 ranks, 2 each, full model width 200, tracking dims).

The parent test fits the same model in one process with a recorded index tape and
saves the result; here each rank fits only ITS members (distributed.MemberShard:
per step only the log-var bound gradients are exchanged) on the same tape, and
after the post-fit member all-gather every rank must hold the single-process
parameters of all 8 members, its losses and its elites. Exit 0 = parity."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def build(dev):
    import numpy as np
    import torch
    import bench
    alg = bench.make_alg(dev, 256, 4, 8, 17, bench.ENV_JSON['tracking'], env='tracking')
    rep = bench.synth_replay('tracking', 6000, np.random.RandomState(2))
    alg.replay_buffer.extend(**{k: torch.from_numpy(v).to(dev) for k, v in rep.items()})
    return alg


def flat_params(m):
    """Every state_dict tensor of the model, flattened in key order (the flat group's
    alignment padding is not a parameter)."""
    import numpy as np
    sd = m.state_dict()
    return np.concatenate([sd[k].detach().cpu().numpy().ravel() for k in sorted(sd)])


def tape(steps, n, rows, hold):
    import numpy as np
    rng = np.random.RandomState(5)
    return [('randint', rng.randint(0, n, rows).astype(np.int64)) for _ in range(steps)] + \
        [('randint', rng.randint(0, n, hold).astype(np.int64))]


def main():
    import numpy as np
    import torch
    import torch.distributed as dist
    out_path = sys.argv[1]
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    torch.set_num_threads(2)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import drpo_amd
    from drpo_amd.distributed import member_sharding
    dev = torch.device('cuda', 0)
    alg = build(dev)
    m = alg.model_ensemble
    sh = member_sharding(m)
    assert sh is not None and sh.count == 2 and sh.even
    if rank > 0:
        m.group.data.add_(0.25 * rank)      # other members must come back through the gather
        ref0 = build(dev).model_ensemble.group.data
        for prefix, spec in m.engine._specs():
            for i in range(spec.n_layers):
                for key in (f'{prefix}{2 * i}.weight', f'{prefix}{2 * i}.bias'):
                    m.group.view(key)[sh.z0:sh.z1].copy_(m.group.view(key, ref0)[sh.z0:sh.z1])
        for key in ('min_log_var', 'max_log_var'):
            m.group.view(key).copy_(m.group.view(key, ref0))
    from drpo_amd.distributed import CommLog
    c0 = CommLog.calls
    losses = m.fit(alg.replay_buffer, steps=3, noise=drpo_amd.TapeNoise(tape(3, len(alg.replay_buffer), 8 * 256, 256)))
    torch.cuda.synchronize()
    # the fused member-shard step (ensemble_engine.fit): ONE all-reduce per fit step (the
    # log-var bounds' gradients) + the per-step loss vector's sum after the fit
    assert m.engine.fit_path == 'fused-shard', m.engine.fit_path
    assert CommLog.calls - c0 == 3 + 1, CommLog.calls - c0
    ref = np.load(out_path)
    np.testing.assert_allclose(losses, ref['losses'], rtol=1e-5)
    assert m._elite_inds == list(ref['elites']), (m._elite_inds, ref['elites'])
    np.testing.assert_allclose(flat_params(m), ref['params'], rtol=1e-5, atol=1e-6)
    dist.barrier()
    dist.destroy_process_group()
    print(f'rank {rank}: member-sharded E=8 fit parity ok')


if __name__ == '__main__':
    main()
