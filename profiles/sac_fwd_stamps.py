"""In-kernel phase timing of the SAC update's multi-job forward launches (profiling
build with s_memtime stamps: DRPO_LIB_OVERRIDE=<...>/libdrpo_hip_stamps.so), config-2
workload (quadrotor, B = 4096, DRPO flags). After one warm rollout_and_update, one
update_solver (critic + actor + multiplier) runs with every drpo_mlp_forward_multi
launch followed by a synchronize and a copy of the stamp buffer, so each launch's
workgroups are read before the next launch overwrites them.

Per launch and (job, net) slot it prints the mean cycles of each phase
(0 start, 1 input staged, 2.. after each layer of a plain net / the trunk, 5 paired
heads' hidden layer, 6 paired heads' output layer, 15 end incl. the fused head) and
the launch's workgroup timeline: the spread of start times and the end of the last
workgroup relative to the first start (cycles)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = {0: 'start', 1: 'staged', 2: 'L0', 3: 'L1', 4: 'L2', 5: 'pair hidden', 6: 'pair out', 15: 'end'}


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
    eng = alg.solver.engine
    orig = eng._run_multi
    n = 1 << 15
    got = []

    def run_multi(key, builder, ctr):
        buf = np.zeros((1 << 16, 16), np.uint64)
        torch.cuda.synchronize()
        L.drpo_debug_stamps_clear()
        orig(key, builder, ctr)
        torch.cuda.synchronize()
        L.drpo_debug_stamps(buf.ctypes.data, n)
        arr, _, nj, _ = eng.desc[key]
        slots = []
        for j in range(nj):
            d = arr[j]
            ns = 1 if d.trunk else d.nnets
            for h in range(ns):
                slots.append((j, h, bool(d.trunk), d.net[h if not d.trunk else 0].nl))
        got.append((key, buf[:n].astype(np.int64).copy(), slots))

    eng._run_multi = run_multi
    alg.update_solver(update_actor=True, update_multiplier=True)
    torch.cuda.synchronize()
    eng._run_multi = orig
    tiles = 256
    for key, st, slots in got:
        nwg = len(slots) * tiles
        st = st[:nwg]
        t0 = st[:, 0]
        live = t0 > 0
        ends = st[:, 15]
        print(f'== {key}: {len(slots)} slots x {tiles} tiles; start spread {t0[live].max() - t0[live].min()} cyc, '
              f'last end {ends.max() - t0[live].min()} cyc after the first start')
        for si, (j, h, trunk, nl) in enumerate(slots):
            s = st[si * tiles:(si + 1) * tiles]
            cols = [c for c in sorted(NAMES) if (s[:, c] > 0).all()]
            parts = []
            for a, b in zip(cols, cols[1:]):
                parts.append(f'{NAMES[b]} {np.mean(s[:, b] - s[:, a]):7.0f}')
            tot = np.mean(s[:, 15] - s[:, 0]) if 15 in cols else float('nan')
            rel0 = np.mean(s[:, 0] - t0[live].min())
            print(f'   slot {si} (job {j}{" trunk" if trunk else f" net {h}"}): start +{rel0:7.0f}  '
                  + ' | '.join(parts) + f'  | total {tot:7.0f}')


if __name__ == '__main__':
    main()
