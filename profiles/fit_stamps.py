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
    L.drpo_debug_stamps_wgrad_clear()
    torch.cuda.synchronize()
    m.fit(alg.replay_buffer, steps=1)
    torch.cuda.synchronize()
    if m.engine.fit_fb:     # the one-launch step (csrc/fit.hip FSTAMP 0..8)
        L.drpo_debug_stamps_fit.argtypes = [ctypes.c_void_p, ctypes.c_int]
        fb = np.zeros((4096, 16), np.uint64)
        L.drpo_debug_stamps_fit(fb.ctypes.data, 4096)
        fb = fb.astype(np.int64)
        fb = fb[fb[:, 0] > 0]
        print(f'== fit_fb_kernel (forward + NLL + backward-data): {len(fb)} workgroups')
        for a, b, name in ((0, 1, 'stage x'), (1, 2, 'trunk L1'), (2, 3, 'trunk L2'), (3, 4, 'heads hidden+out'),
                           (4, 5, 'NLL'), (5, 6, 'B1 head out^T'), (6, 7, 'B2 head hidden^T'), (7, 8, 'B3 trunk L2^T'),
                           (0, 9, ' preloads'), (9, 1, ' staging'), (1, 10, ' L1 mma'), (10, 11, ' L1 next prefetch'),
                           (11, 12, ' L1 epilogue'), (12, 2, ' L1 barrier'), (5, 13, ' B1 mma'),
                           (13, 14, ' B1 next prefetch'), (14, 15, ' B1 epilogue'), (15, 6, ' B1 barrier')):
            if fb[:, b].max() == 0 or fb[:, a].max() == 0:
                continue
            d = fb[:, b] - fb[:, a]
            print(f'   {name:20s} mean {d.mean():8.0f} min {d.min():8.0f} max {d.max():8.0f} cyc')
        d = fb[:, 8] - fb[:, 0]
        print(f'   workgroup total       mean {d.mean():8.0f} min {d.min():8.0f} max {d.max():8.0f} cyc')
        t0 = fb[:, 0].min()
        wgrad_phases(L)
        return
    L.drpo_debug_stamps(buf.ctypes.data, n)
    # forward (mlp_fwd_kernel STAMP rows 0..: 0 start, 1 input staged, 2/3 trunk layers,
    # 6/7 head 1 layers (lb.y == 0), 10/11 head 2 layers (lb.y == 1))
    fw = buf[0:4096].astype(np.int64)
    nf = int((fw[:, 0] > 0).sum())
    fw = fw[:nf]
    print(f'== mlp_fwd_kernel (fit step, split heads): {nf} workgroups')
    for a, b, name in ((0, 1, 'stage input'), (1, 2, 'trunk L1'), (2, 3, 'trunk L2'), (3, 6, 'head1 L1'),
                       (6, 7, 'head1 L2'), (3, 10, 'head2 L1'), (10, 11, 'head2 L2')):
        ok = (fw[:, a] > 0) & (fw[:, b] > 0)
        if ok.any():
            d = fw[ok, b] - fw[ok, a]
            print(f'   {name:20s} mean {d.mean():8.0f} min {d.min():8.0f} max {d.max():8.0f} cyc  (n={ok.sum()})')
    end = np.maximum(fw[:, 7], fw[:, 11])
    d = end - fw[:, 0]
    print(f'   workgroup total       mean {d.mean():8.0f} min {d.min():8.0f} max {d.max():8.0f} cyc')
    bw = buf[32768:32768 + 4096].astype(np.int64)
    nb = int((bw[:, 0] > 0).sum())
    bw = bw[:nb]
    split = nb > 0 and bw[:, 3].max() == 0     # split heads: stamps 0, 1, 2, 12 only
    print(f'== mlp_bwd_ens_kernel (fit step, {"split" if split else "paired"} heads + NLL upstream): {nb} workgroups')
    phases = (((0, 1, 'NLL upstream'), (1, 2, 'head backward'), (2, 12, 'trunk share backward')) if split else
              ((0, 5, ' start -> NLL loop'), (5, 6, ' NLL element loop'), (6, 7, ' mse wave sums'),
               (7, 1, ' partials + barrier'), (0, 1, 'NLL upstream'), (1, 2, 'heads out bwd'),
               (2, 3, 'hidden act grad'), (3, 4, 'heads -> trunk catK'), (4, 12, 'trunk backward')))
    for a, b, name in phases:
        ok = (bw[:, a] > 0) & (bw[:, b] > 0)
        if ok.any():
            d = bw[ok, b] - bw[ok, a]
            print(f'   {name:20s} mean {d.mean():8.0f} min {d.min():8.0f} max {d.max():8.0f} cyc  (n={ok.sum()})')
    ok = bw[:, 12] > 0
    if ok.any():
        d = bw[ok, 12] - bw[ok, 0]
        print(f'   workgroup total       mean {d.mean():8.0f} min {d.min():8.0f} max {d.max():8.0f} cyc')

def wgrad_phases(L):
    """the step's weight-gradient + Adam launch (csrc/wgrad.hip STAMPG 0..5)"""
    L.drpo_debug_stamps_wgrad.argtypes = [ctypes.c_void_p, ctypes.c_int]
    st = np.zeros((1 << 14, 8), np.uint64)
    L.drpo_debug_stamps_wgrad(st.ctypes.data, 1 << 14)
    st = st.astype(np.int64)
    st = st[st[:, 0] > 0]
    print(f'== mlp_wgrad_kernel (+ Adam): {len(st)} workgroups')
    for a, b, name in ((0, 6, 'setup'), (6, 7, 'first k-group'), (7, 5, 'next 3 k-groups'), (0, 5, 'ring fill'), (0, 1, 'main loop'), (1, 2, 'lds reduce'), (2, 3, 'slab + ticket'),
                       (3, 4, 'last finish'), (2, 4, 'finish (adam)'), (0, 4, 'total')):
        ok = (st[:, a] > 0) & (st[:, b] > 0)
        if ok.any():
            d = st[ok, b] - st[ok, a]
            print(f'   {name:20s} mean {d.mean():8.0f} min {d.min():8.0f} p90 {np.percentile(d, 90):8.0f} '
                  f'max {d.max():8.0f} cyc  (n={ok.sum()})')


if __name__ == '__main__':
    main()
