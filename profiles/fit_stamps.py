"""In-kernel phase timing of the model fit's mlp_wgrad_kernel (profiling build with
s_memtime stamps, DRPO_LIB_OVERRIDE=<...>/libdrpo_hip_stamps.so): per-workgroup
cycles in each phase and the spread of workgroup start / end times."""
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
    cd = bench.CONFIGS[2]
    dev = torch.device('cuda')
    alg = bench.make_alg(dev, 256, cd['H'], cd['E'], 0, bench.ENV_JSON[cd['env']], env=cd['env'])
    rep = bench.synth_replay(cd['env'], 100000, np.random.RandomState(0))
    alg.replay_buffer.extend(**{k: torch.from_numpy(v).to(dev) for k, v in rep.items()})
    m = alg.model_ensemble
    m.fit(alg.replay_buffer, steps=5)
    torch.cuda.synchronize()
    n = 1 << 16
    buf = np.zeros((n, 16), np.uint64)
    m.fit(alg.replay_buffer, steps=1)
    torch.cuda.synchronize()
    L.drpo_debug_stamps(buf.ctypes.data, n)
    st = buf[32768:32768 + 4096, 0:5].astype(np.int64)   # STAMPW rows (csrc/mlp.hip)
    nwg = int((st[:, 4] > 0).sum())
    st = st[:nwg]
    t0 = st[:, 0].min()
    print(f'== mlp_wgrad_kernel (fit step, config 2): {nwg} workgroups')
    print(f'   start offsets (cycles) pct 0/25/50/75/100: {np.percentile(st[:, 0] - t0, [0, 25, 50, 75, 100]).astype(int)}')
    print(f'   end offsets   (cycles) pct 0/25/50/75/100: {np.percentile(st[:, 4] - t0, [0, 25, 50, 75, 100]).astype(int)}')
    names = ['first stage loaded', 'stage loop', 'wave reduce', 'atomics + bias']
    for c in range(1, 5):
        d = st[:, c] - st[:, c - 1]
        print(f'   {names[c - 1]:20s} mean {d.mean():8.0f} min {d.min():8.0f} max {d.max():8.0f} cyc')
    d = st[:, 4] - st[:, 0]
    print(f'   workgroup total       mean {d.mean():8.0f} min {d.min():8.0f} max {d.max():8.0f} cyc')
    bw = buf[32768:32768 + 4096, 5:14].astype(np.int64)
    nb = int((bw[:, 8] > 0).sum())
    bw = bw[:nb]
    print(f'== mlp_bwd_kernel (fit step, trunk + 2 heads): {nb} workgroups')
    names = ['head 1 gout load', 'head 1 backward', 'head 1 add to dT', 'head 2 gout load', 'head 2 backward',
             'head 2 add to dT', 'trunk backward', 'dx store']
    for c in range(1, 9):
        d = bw[:, c] - bw[:, c - 1]
        print(f'   {names[c - 1]:20s} mean {d.mean():8.0f} min {d.min():8.0f} max {d.max():8.0f} cyc')
    d = bw[:, 8] - bw[:, 0]
    print(f'   workgroup total       mean {d.mean():8.0f} min {d.min():8.0f} max {d.max():8.0f} cyc')


if __name__ == '__main__':
    main()
