"""Model-fit micro-benchmark (bench config 2 shapes: E=7, 256 rows per member, model
width 200): wall time per fit step and, under rocprofv3, the kernels of the step."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    c = int(os.environ.get('FIT_CONFIG', '2'))
    cd = bench.CONFIGS[c]
    dev = torch.device('cuda')
    alg = bench.make_alg(dev, 256, cd['H'], cd['E'], 0, bench.ENV_JSON[cd['env']], env=cd['env'])
    rep = bench.synth_replay(cd['env'], 100000, np.random.RandomState(0))
    alg.replay_buffer.extend(**{k: torch.from_numpy(v).to(dev) for k, v in rep.items()})
    m = alg.model_ensemble
    m.fit(alg.replay_buffer, steps=5)
    torch.cuda.synchronize()
    steps = int(os.environ.get('FIT_STEPS', '300'))
    t0 = time.perf_counter()
    m.fit(alg.replay_buffer, steps=steps)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    print(f'config {c}: {dt * 1e3:.4f} ms per fit step ({steps} steps)')


if __name__ == '__main__':
    main()
