"""Per-launch timing of the SAC update's MLP kernels (HIP events around each launch)
on the bench workload (quadrotor, B=4096, DRPO flags). Prints one JSON object:
{kind[:descriptor]: {launches, ms, avg_ms, flop, tflops}}.

    python profiles/sac_micro.py [--steps 5] [--batch 4096]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from drpo_amd.sac_step import LaunchProfiler
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--batch', type=int, default=4096)
    args, _ = ap.parse_known_args()
    dev = torch.device('cuda')
    B = args.batch
    alg = bench.make_alg(dev, B, 10, 7, 0, bench.QUAD_JSON)
    rep = bench.synth_replay('quadrotor', 100000, np.random.RandomState(0))
    alg.replay_buffer.extend(**{k: torch.from_numpy(v).to(dev) for k, v in rep.items()})
    alg.model_ensemble.state_normalizer.fit(alg.replay_buffer.get('states'))
    bench.steady_mode(alg)
    for _ in range(3):
        alg.rollout_and_update()
    torch.cuda.synchronize()
    eng = alg.solver.engine
    eng.profiler = LaunchProfiler()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.steps):
        for st in range(alg.solver_updates_per_step):
            alg.update_solver(update_actor=st % 2 == 0, update_multiplier=st % 5 == 0)
    e1.record()
    torch.cuda.synchronize()
    out = eng.profiler.summarise()
    out['_total'] = {'updates': args.steps * alg.solver_updates_per_step, 'ms': e0.elapsed_time(e1),
                     'ms_per_update': e0.elapsed_time(e1) / (args.steps * alg.solver_updates_per_step)}
    eng.profiler = None
    print(json.dumps(out))


if __name__ == '__main__' and '--host' not in sys.argv:
    main()


def host_vs_gpu(steps=20):
    """Host enqueue time vs GPU time per update_solver (is the update host-bound?)."""
    import time
    import bench
    dev = torch.device('cuda')
    alg = bench.make_alg(dev, 4096, 10, 7, 0, bench.QUAD_JSON)
    rep = bench.synth_replay('quadrotor', 100000, np.random.RandomState(0))
    alg.replay_buffer.extend(**{k: torch.from_numpy(v).to(dev) for k, v in rep.items()})
    alg.model_ensemble.state_normalizer.fit(alg.replay_buffer.get('states'))
    bench.steady_mode(alg)
    for _ in range(3):
        alg.rollout_and_update()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(steps):
        for st in range(alg.solver_updates_per_step):
            alg.update_solver(update_actor=st % 2 == 0, update_multiplier=st % 5 == 0)
    e1.record()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    n = steps * alg.solver_updates_per_step
    print(json.dumps({'host_enqueue_ms_per_update': (t1 - t0) * 1e3 / n, 'gpu_ms_per_update': e0.elapsed_time(e1) / n,
                      'wall_ms_per_update': (t2 - t0) * 1e3 / n}))


if __name__ == '__main__' and '--host' in sys.argv:
    host_vs_gpu()
