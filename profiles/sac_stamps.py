"""In-kernel phase timing of the SAC critic update's backward launch (profiling build
with s_memtime stamps, DRPO_LIB_OVERRIDE=<...>/libdrpo_hip_stamps.so), config-2
workload: the constraint critic's workgroups (grid slot 0: certificate upstream, paired
heads, trunk) and the twin critics' (slots 1-2, stamp 0 to the end of the launch is not
stamped; their start spread is printed)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from drpo_amd import _lib
    L = _lib.lib()
    L.drpo_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device('cuda')
    alg = bench.make_alg(dev, 4096, 10, 7, 0, bench.QUAD_JSON)
    rep = bench.synth_replay('quadrotor', 100000, np.random.RandomState(0))
    alg.replay_buffer.extend(**{k: torch.from_numpy(v).to(dev) for k, v in rep.items()})
    alg.model_ensemble.state_normalizer.fit(alg.replay_buffer.get('states'))
    bench.steady_mode(alg)
    alg.rollout_and_update()
    torch.cuda.synchronize()
    # one critic-only update: its backward is the last backward launch before the read
    alg.update_solver(update_actor=False, update_multiplier=False)
    torch.cuda.synchronize()
    n = 1 << 16
    buf = np.zeros((n, 16), np.uint64)
    L.drpo_debug_stamps(buf.ctypes.data, n)
    bw = buf[32768:32768 + 768].astype(np.int64)
    cc = bw[:256]
    print('== mlp_bwd_multi_kernel<critic> (config 2, B = 4096): constraint-critic workgroups (slot 0)')
    for a, b, name in ((0, 1, 'cert upstream'), (1, 2, 'heads out bwd'), (2, 3, 'hidden act grad'),
                       (3, 4, 'heads -> trunk catK'), (4, 12, 'trunk backward'), (0, 12, 'workgroup total')):
        ok = (cc[:, a] > 0) & (cc[:, b] > 0)
        if ok.any():
            d = cc[ok, b] - cc[ok, a]
            print(f'   {name:20s} mean {d.mean():8.0f} min {d.min():8.0f} max {d.max():8.0f} cyc  (n={ok.sum()})')


if __name__ == '__main__':
    main()
