"""Noise sources for the hot path.

Production: ``DeviceNoise`` -- kernels draw Philox4x32-10 normals / uniforms on
the device from (seed, per-call counter, call-site id); host-RNG choices the
reference makes on the host (elite member per rollout step, critic pick) keep
using Python's ``random`` like the reference.

Parity mode: ``TapeNoise`` -- replays a recorded draw sequence (the format of
tests/golden/tape.py) in the reference's call order, so the HIP path consumes
exactly the random numbers the reference consumed (noise injection).
"""
import random

import numpy as np


def _mix64(x):
    """splitmix64 finaliser: decorrelates Philox keys derived from (seed, rank)."""
    x = (x + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return x ^ (x >> 31)


class DeviceNoise:
    """Production noise.

    * Device draws (Philox4x32-10) are keyed by ``seed``: the base seed on rank 0 and
      a splitmix64 mix of (base seed, rank) on the other data-parallel ranks, so each
      rank draws its own minibatches, initial states and Gaussian noise.
    * Host choices the reference makes with Python's ``random`` (elite member per
      rollout step, src/dynamics.py:199; critic pick, src/ssac.py:43) come from a
      private ``random.Random(base seed)`` that is identical on every rank: all
      replicas pick the same member / critic, so the mean-all-reduced gradient is
      the gradient of one well-defined loss.

    ``seed=None`` takes ``torch.initial_seed()`` (what set_seed / torch.manual_seed
    set, src/util.py:11-17) of rank 0, broadcast to every rank when the job is data
    parallel (a driver that seeds torch per rank, seed + rank, still gets one shared
    host stream; constructing with seed=None is then a collective call). An explicit
    ``seed`` must be equal on all ranks. ``rank=None`` takes the torch.distributed rank."""
    parity = False
    COLLECT_SALT = 0xC011EC7ED

    def __init__(self, seed=None, rank=None, world=None):
        from . import distributed as dist
        if seed is None:
            import torch
            seed = dist.broadcast_int(torch.initial_seed())
        if rank is None:
            rank = dist.rank()
        self.base_seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.rank = int(rank)
        self.world = dist.world_size() if world is None else int(world)
        self.seed = self.base_seed if self.rank == 0 else _mix64(self.base_seed ^ _mix64(self.rank))
        self.host = random.Random(self.base_seed)
        self.ctr = 0
        self._collect = None

    def collection(self):
        """Noise for the real-env collection (uniform warm-up and actor actions, the
        safety shield's critic draw; src/smbpo.py:124-136). Single process: this
        stream. Data parallel: a stream keyed by the base seed only, identical on every
        rank, so every replica collects the same real transitions (with identically
        seeded envs) and fits the same normalizer and reward bounds."""
        if self.world <= 1:
            return self
        if self._collect is None:
            self._collect = DeviceNoise(_mix64(self.base_seed ^ self.COLLECT_SALT), rank=0, world=1)
        return self._collect

    def next(self):
        self.ctr += 1
        return self.ctr

    # reference host-RNG call sites (shared across ranks)
    def choice(self, n):
        return self.host.choice(range(n))

    # device-drawn sites: nothing to hand over
    def np_choice(self, high, size):
        return None

    def normal(self, shape):
        return None

    def std_normal(self, shape):
        return None

    def randn_like(self, shape, used=True):
        return None

    def randint(self, high, n):
        return None

    def rand(self, shape):
        """Uniform [0, 1) draws of the warm-up UniformPolicy (src/policy.py:43-47): a host
        Philox stream keyed by (seed, per-call counter) -- one action row per real step,
        and the same on every rank for the collection stream."""
        g = np.random.Generator(np.random.Philox(key=self.seed, counter=self.next()))
        return g.random(shape, dtype=np.float32)


class TapeNoise:
    parity = True

    def __init__(self, entries):
        self.entries = list(entries)
        self.pos = 0
        self.seed, self.ctr = 0, 0

    @classmethod
    def from_npz(cls, d, prefix):
        n = int(d[f'{prefix}_n'])
        keys = sorted(k for k in d.files if k.startswith(prefix + '_') and k != f'{prefix}_n')
        assert len(keys) == n
        return cls([(k[len(prefix) + 6:], d[k]) for k in keys])

    def next(self):
        return 0

    def collection(self):
        return self

    def peek(self):
        return self.entries[self.pos][0] if self.pos < len(self.entries) else None

    def _take(self, kind, shape=None):
        if self.pos >= len(self.entries):
            raise AssertionError(f'noise tape exhausted (wanted {kind})')
        k, v = self.entries[self.pos]
        if k != kind:
            raise AssertionError(f'noise tape position {self.pos}: expected {kind}, found {k}')
        if shape is not None and tuple(v.shape) != tuple(shape):
            raise AssertionError(f'noise tape {kind} shape {v.shape} != {tuple(shape)}')
        self.pos += 1
        return v

    def choice(self, n):
        return int(self._take('choice'))

    def np_choice(self, high, size):
        return np.asarray(self._take('np_choice', (size,)), dtype=np.int64)

    def normal(self, shape):
        return np.ascontiguousarray(self._take('normal', shape), dtype=np.float32)

    def std_normal(self, shape):
        return np.ascontiguousarray(self._take('normal_', shape), dtype=np.float32)

    def randn_like(self, shape, used=True):
        return np.ascontiguousarray(self._take('randn_like', shape), dtype=np.float32)

    def randint(self, high, n):
        return np.asarray(self._take('randint', (n,)), dtype=np.int64)

    def rand(self, shape):
        return np.ascontiguousarray(self._take('rand', shape), dtype=np.float32)

    def done(self):
        return self.pos == len(self.entries)
