"""Host-side enqueue cost of the hot-path calls against their GPU time (config 2 shapes).

For each call kind it times (a) the host wall time to ENQUEUE n calls with the GPU
kept busy (a long spin of prior work in the queue, no synchronisation in between),
and (b) the GPU time of the same n calls (events around them). Host > GPU means
the stream starves and the phase timings include host latency.

Usage: python profiles/host_probe.py [--config 2] [--n 50]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', type=int, default=2)
    ap.add_argument('--n', type=int, default=50)
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    cfgd = bench.CONFIGS[args.config]
    env = cfgd['env']
    alg = bench.make_alg(dev, cfgd['B'], cfgd['H'], cfgd['E'], 0, bench.ENV_JSON[env], env=env)
    rep = bench.synth_replay(env, 100000, np.random.RandomState(0), dev, alg.env_params)
    alg.replay_buffer.extend(**{k: torch.from_numpy(v).to(dev) for k, v in rep.items()})
    alg.model_ensemble.state_normalizer.fit(alg.replay_buffer.get('states'))
    bench.steady_mode(alg)
    calls = {
        'rollout': lambda i: alg.rollout(alg.actor),
        'update_solver': lambda i: alg.update_solver(update_actor=i % 2 == 0, update_multiplier=i % 5 == 0),
    }
    big = torch.empty(1 << 28, device=dev)
    out = {}
    for name, fn in calls.items():
        for i in range(5):
            fn(i)
        torch.cuda.synchronize()
        # GPU time
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(args.n):
            fn(i)
        e1.record()
        torch.cuda.synchronize()
        gpu_ms = e0.elapsed_time(e1) / args.n
        # host enqueue time with a busy queue in front
        for _ in range(40):
            big.mul_(1.0000001)     # ~40 x 0.35 ms of HBM streaming ahead of the calls
        t0 = time.perf_counter()
        for i in range(args.n):
            fn(i)
        host_ms = (time.perf_counter() - t0) * 1e3 / args.n
        torch.cuda.synchronize()
        out[name] = {'host_enqueue_ms': round(host_ms, 4), 'gpu_ms': round(gpu_ms, 4)}
    print(json.dumps(out))


if __name__ == '__main__':
    main()
