"""In-kernel phase timing of mlp_fwd_kernel (profiling build with s_memtime stamps).
Runs with DRPO_LIB_OVERRIDE=<...>/libdrpo_hip_stamps.so. For each case prints the
per-workgroup cycles spent in each phase (input staging, each layer) and the
spread of workgroup start / end times across the grid."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    import drpo_amd
    from drpo_amd import _lib, ops
    L = _lib.lib()
    L.drpo_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device('cuda')
    alg = bench.make_alg(dev, 4096, 10, 7, 0, bench.QUAD_JSON)
    sol = alg.solver
    s = torch.randn(4096, 12, device=dev)
    a = torch.rand(4096, 2, device=dev) * 2 - 1
    cases = {
        'actor 12-256-256-4': lambda: ops.policy_raw(sol.actor, s),
        'twin critic 14-256-256-1 x2': lambda: sol.critic.all(s, a),
        'cc trunk+2 heads': lambda: sol.constraint_critic(s, a, uncertainty=True),
    }
    buf = np.zeros((1 << 16, 16), np.uint64)
    for name, fn in cases.items():
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        L.drpo_debug_stamps(ctypes.c_void_p(0), 0)
        fn()
        torch.cuda.synchronize()
        L.drpo_debug_stamps(buf.ctypes.data, 1 << 16)
        st = buf.astype(np.int64)
        nwg = int((st[:, 0] > 0).sum())
        st = st[:nwg]
        t0 = st[:, 0]
        print(f'== {name}: {nwg} workgroups')
        print(f'   start spread {t0.max() - t0.min()} cyc; total span {st.max() - t0.min()} cyc')
        cols = [c for c in range(1, 16) if (st[:, c] > 0).all()]
        prev = 0
        for c in cols:
            d = st[:, c] - st[:, prev]
            print(f'   phase {prev}->{c}: mean {d.mean():8.0f} min {d.min():8.0f} max {d.max():8.0f} cyc')
            prev = c
        buf[:] = 0


if __name__ == '__main__' and not os.environ.get('DRPO_STAMPS_ROLLOUT'):
    main()


def rollout_stamps():
    """Phase timing of rollout_step_kernel (step 1 of a steady-mode bench rollout)."""
    import bench
    from drpo_amd import _lib
    L = _lib.lib()
    L.drpo_debug_stamps_rollout.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device('cuda')
    alg = bench.make_alg(dev, 4096, 10, 7, 0, bench.QUAD_JSON)
    rep = bench.synth_replay('quadrotor', 100000, np.random.RandomState(0))
    alg.replay_buffer.extend(**{k: torch.from_numpy(v).to(dev) for k, v in rep.items()})
    alg.model_ensemble.state_normalizer.fit(alg.replay_buffer.get('states'))
    bench.steady_mode(alg)
    alg.horizon = int(os.environ.get('DRPO_STAMPS_H', '1'))   # stamps keep the last step's launch
    alg.rollout_engine = 1
    for _ in range(3):
        alg.rollout(alg.actor)
    torch.cuda.synchronize()
    buf = np.zeros((1 << 14, 16), np.uint64)
    L.drpo_debug_stamps_rollout(buf.ctypes.data, 256)
    st = buf[:256].astype(np.int64)
    names = ['scan', 'gather', 'actor L1', 'actor L2', 'actor L3', 'sample', 'member L1', 'member L2', 'diff L1',
             'diff L2', 'lv L1', 'lv L2', 'gauss', 'constraints', 'writes']
    print('== rollout_step_kernel (B=4096, quadrotor): cycles per phase, mean over 256 workgroups')
    tot = 0
    for c in range(1, 15):
        d = st[:, c] - st[:, c - 1]
        tot += d.mean()
        print(f'   {names[c]:12s} mean {d.mean():8.0f} min {d.min():8.0f} max {d.max():8.0f}')
    print(f'   total {tot:.0f} cycles')


def fused_stamps():
    """Phase timing of rollout_persist_kernel (horizon step t=2 of a bench rollout)."""
    import bench
    from drpo_amd import _lib
    L = _lib.lib()
    L.drpo_debug_stamps_rollout.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device('cuda')
    hm = int(os.environ.get('DRPO_STAMPS_HM', '200'))   # model width (200 = reference; else the unpaired path)
    c = int(os.environ.get('DRPO_STAMPS_CONFIG', '2'))   # BASELINE config (bench.CONFIGS)
    cd = bench.CONFIGS[c]
    env = cd['env']
    # DRPO_STAMPS_H=3: the layer cores' sub-phase stamps (slots 11-15, written every
    # step) then come from the same step t = 2 as the phase stamps
    hz = min(cd['H'], int(os.environ.get('DRPO_STAMPS_H', '10')))
    alg = bench.make_alg(dev, cd['B'], hz, cd['E'], 0, bench.ENV_JSON[env],
                         extra={'model_cfg': {'hidden_dim': hm}}, env=env)
    rep = bench.synth_replay(env, 100000, np.random.RandomState(0))
    alg.replay_buffer.extend(**{k: torch.from_numpy(v).to(dev) for k, v in rep.items()})
    alg.model_ensemble.state_normalizer.fit(alg.replay_buffer.get('states'))
    bench.steady_mode(alg)
    if os.environ.get('DRPO_STAMPS_ONE_MEMBER'):      # every step on member 0 (L2-warm member weights)
        alg.model_ensemble._elite_inds = [0]
    alg.rollout_engine = 2
    for _ in range(3):
        alg.rollout(alg.actor)
    torch.cuda.synchronize()
    buf = np.zeros((1 << 14, 16), np.uint64)
    L.drpo_debug_stamps_rollout(buf.ctypes.data, 256)
    st = buf[:256].astype(np.int64)
    names = ['start', 'noise', 'actor L1', 'actor L2', 'actor L3+sample', 'member L1', 'member L2', 'pair L1',
             'pair L2+gauss', 'constr+staging']
    if hm != 200:
        names[7:9] = ['diff L1+L2, lv L1', 'lv L2, gauss']
    elif env == 'tracking':
        names[7:9] = ['pair L1', 'pair L2 (2 inputs) + gauss']
    print(f'== rollout_persist_kernel step t=2 (config {c}: {env} B={cd["B"]} E={cd["E"]}): cycles per phase, '
          'mean over the first 256 workgroups')
    tot = 0
    for c in range(1, len(names)):
        d = st[:, c] - st[:, c - 1]
        tot += d.mean()
        print(f'   {names[c]:12s} mean {d.mean():8.0f} min {d.min():8.0f} max {d.max():8.0f}')
    print(f'   total {tot:.0f} cycles')
    if hz == 3 and (st[:, 11] > 0).all() and (st[:, 13] > 0).all():
        m = lambda a, b: (st[:, b] - st[:, a]).mean()   # noqa: E731
        print(f'   pair L1 wave 0 (4 blocks): k-loop issued {m(6, 13):.0f} | epilogue {m(13, 14):.0f} | '
              f'output partials {m(14, 15):.0f} | barrier {m(15, 7):.0f}')
        print(f'   pair L1 wave 4 (3 blocks, same SIMD): k-loop issued {m(6, 11):.0f} | epilogue {m(11, 12):.0f}')
    if env == 'tracking' and (st[:, 10] > 0).all():
        d = st[:, 10] - st[:, 7]
        print(f'   (of pair L2 + gauss: output layers {d.mean():.0f}, gauss {(st[:, 8] - st[:, 10]).mean():.0f})')


if __name__ == '__main__' and os.environ.get('DRPO_STAMPS_ROLLOUT') == 'fused':
    fused_stamps()
elif __name__ == '__main__' and os.environ.get('DRPO_STAMPS_ROLLOUT'):
    rollout_stamps()
