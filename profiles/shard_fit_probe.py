"""Per-rank cost of the member-sharded model fit on ONE GPU (no collective: the
MemberShard's exchanges are stubbed out, so this is the rank's own GPU work, the
shape config 4 gives each of its 4 ranks: E = 8 tracking members, 2 per rank, width
200, 256 rows per member) against the single-process fused fit of the same members.

    python profiles/shard_fit_probe.py [--steps 300]

Prints one JSON object: ms per fit step for
  shard_e8_rank0   members [0, 2) of E = 8 through the member-shard path
  single_e2        an E = 2 model through the single-process fused path
  single_e8        the whole E = 8 model, single process
and the fit path each took (ensemble_engine.fit_path)."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    import drpo_amd.distributed as D
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=300)
    args = ap.parse_args()
    dev = torch.device('cuda')

    class StubShard(D.MemberShard):
        """rank 0 of a 4-rank member shard, exchanges stubbed (one GPU, one process)"""

        def sum_(self, t):
            pass

        def broadcast_(self, *ts, src=0):
            pass

        def gather_members_(self, t):
            return t

    def timed(E, shard):
        alg = bench.make_alg(dev, 256, 40, E, 3, bench.ENV_JSON['tracking'], env='tracking')
        rep = bench.synth_replay('tracking', 30000, np.random.RandomState(1))
        alg.replay_buffer.extend(**{k: torch.from_numpy(v).to(dev) for k, v in rep.items()})
        m = alg.model_ensemble
        orig = D.member_sharding
        if shard:
            D.member_sharding = lambda model: StubShard(model.ensemble_size, world=4, rank_=0)
        try:
            m.fit(alg.replay_buffer, steps=5)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            m.fit(alg.replay_buffer, steps=args.steps)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / args.steps
        finally:
            D.member_sharding = orig
        return {'ms_per_fit_step': dt * 1e3, 'fit_path': m.engine.fit_path}

    out = {'shard_e8_rank0': timed(8, True), 'single_e2': timed(2, False), 'single_e8': timed(8, False),
           'steps': args.steps}
    print(json.dumps(out))


if __name__ == '__main__':
    main()
