"""Data parallelism for the hot path.

One process per GPU (torchrun), ``torch.distributed`` over RCCL/xGMI ("nccl") or
gloo for the CPU tests. The path shards with ONE exchange per optimizer step:

  SAC update   each rank draws its own minibatch shard; after the fused backward
               + weight-gradient kernels, ONE buffer per optimizer phase is
               sum-all-reduced (critic + constraint critic 1.37 MB | the actor
               exchange arena: actor + safe actor gradients + alpha-loss sum,
               0.56 MB | multiplier), then every rank runs the identical clip + Adam
               (the 1/G and the clip on the post-reduce norm ride in the optimizer).
  model fit    same for the ensemble's flat group; the holdout MSEs are averaged
               too so every rank picks the same elites.
  rollout      batch-sharded, no communication inside the horizon loop.

Flat parameter groups make each exchange a single contiguous buffer: no
bucketing logic is needed, and the tiny buffers (<1.4 MB) are latency-bound on
xGMI rings, so one call per group is the right granularity.
"""
import torch

try:
    import torch.distributed as _dist
except ImportError:          # pragma: no cover
    _dist = None


def is_active():
    return _dist is not None and _dist.is_available() and _dist.is_initialized() and _dist.get_world_size() > 1


def world_size():
    return _dist.get_world_size() if is_active() else 1


def rank():
    return _dist.get_rank() if is_active() else 0


class CommLog:
    """Process-wide tally of the data-parallel collectives the hot path issues (tests
    count them per update) and, when ``timing`` is a list, HIP events around each one
    on the current stream (bench.py reports the communication time per update / fit
    step from them in an untimed post-pass)."""
    calls = 0
    timing = None

    @classmethod
    def all_reduce(cls, t, group=None):
        cls.calls += 1
        if cls.timing is not None and t.is_cuda:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            _dist.all_reduce(t, group=group)
            e1.record()
            cls.timing.append((e0, e1))
        else:
            _dist.all_reduce(t, group=group)

    @classmethod
    def take_ms(cls):
        """Sum of the recorded exchange times (ms; call after a synchronize) and reset."""
        ms = sum(a.elapsed_time(b) for a, b in (cls.timing or []))
        if cls.timing is not None:
            cls.timing = []
        return ms


def broadcast_int(value, src=0):
    """Rank ``src``'s value of a 64-bit integer on every rank (identity when not data
    parallel). The tensor lives where the backend exchanges: the GPU for RCCL."""
    if not is_active():
        return value
    v = int(value) & 0xFFFFFFFFFFFFFFFF
    v = v - (1 << 64) if v >= (1 << 63) else v
    dev = torch.device('cuda', torch.cuda.current_device()) if _dist.get_backend() == 'nccl' else 'cpu'
    t = torch.tensor([v], dtype=torch.int64, device=dev)
    _dist.broadcast(t, src)
    return int(t.item()) & 0xFFFFFFFFFFFFFFFF


class GradReducer:
    """Mean all-reduce of flat gradient buffers across the data-parallel ranks."""

    def __init__(self, group=None):
        self.group = group
        self.world = world_size()

    @property
    def active(self):
        return self.world > 1

    @property
    def scale(self):
        """1/G: the factor that turns a sum_() result into the mean. The SAC and fit
        steps hand it to the fused optimizer (drpo_optim_seg_t.grad_scale), which
        applies it to the gradient and to its clip norm in the same pass."""
        return 1.0 / self.world

    def sum_(self, *tensors):
        """Sum all-reduce of flat buffers (the mean's 1/G is left to the consumer)."""
        if self.world == 1:
            return
        for t in tensors:
            if t is not None:
                CommLog.all_reduce(t, group=self.group)

    def mean_(self, *tensors):
        if self.world == 1:
            return
        # sum + scale on every backend (RCCL and gloo run the same code path; the
        # scale is one elementwise pass over <= 1.5 MB)
        for t in tensors:
            if t is None:
                continue
            CommLog.all_reduce(t, group=self.group)
            t.div_(self.world)

    def broadcast_(self, *tensors, src=0):
        if self.world == 1:
            return
        for t in tensors:
            _dist.broadcast(t, src, group=self.group)


def sync_parameters(alg, src=0):
    """Make every rank start from rank ``src``'s parameters (flat groups, targets,
    normalizer, log_alpha): one broadcast per flat buffer."""
    if not is_active():
        return
    red = GradReducer()
    sol, m = alg.solver, alg.model_ensemble
    red.broadcast_(sol.actor.group.data, sol.actor_safe.group.data, sol.critic_group.data,
                   sol.critic_target_group.data, sol.multiplier_group.data, sol.log_alpha, m.group.data,
                   m.state_normalizer.mean, m.state_normalizer.std, src=src)
    for g in (sol.actor.group, sol.actor_safe.group, sol.critic_group, sol.critic_target_group, sol.multiplier_group,
              m.group):
        g.mark_dirty()


class MemberShard:
    """Ensemble-sharded model fit (SURVEY.md §8(e) "model fit"): rank r trains the
    members [z0, z1) of the E-member ensemble. Members are independent except for

      * the shared soft log-var bounds (min/max_log_var, 2(S+1) floats): their
        gradients are sum-all-reduced every step (the bound term's own gradient
        is added by rank 0 only);
      * the holdout MSEs: every rank scores its own members on the SAME holdout
        rows (broadcast from rank 0), then one sum-all-reduce of an [E] vector
        gives every rank the identical argsort -> identical elites;
      * after the fit every rank needs every member for rollouts: one all-gather
        per [E, out, in] layer tensor (members are the leading dimension, so a
        shard is one contiguous slice), broadcasts from each owner when E does
        not divide evenly.

    Per step this exchanges 2(S+1) floats instead of the whole ensemble gradient
    (quadrotor E=32: 19.5 MB), and the per-step algorithm is exactly the
    reference's (each member sees its own 256 rows of the E*256 draw)."""

    def __init__(self, E, world=None, rank_=None, group=None):
        self.E = E
        self.world = world_size() if world is None else world
        self.rank = rank() if rank_ is None else rank_
        self.group = group
        base, rem = divmod(E, self.world)
        self.ranges = []
        z = 0
        for r in range(self.world):
            c = base + (1 if r < rem else 0)
            self.ranges.append((z, z + c))
            z += c
        self.z0, self.z1 = self.ranges[self.rank]

    @property
    def count(self):
        return self.z1 - self.z0

    @property
    def even(self):
        return self.E % self.world == 0

    def sum_(self, t):
        if self.world > 1:
            CommLog.all_reduce(t, group=self.group)

    def broadcast_(self, *ts, src=0):
        if self.world > 1:
            for t in ts:
                _dist.broadcast(t, src, group=self.group)

    def merge_members(self, part, full):
        """part [count, ...] (this rank's members) -> full [E, ...] on every rank."""
        full[self.z0:self.z1].copy_(part)
        self.gather_members_(full)
        return full

    def gather_members_(self, t):
        """t [E, ...]: every rank's own slice -> replicated on all ranks (in place)."""
        if self.world == 1:
            return t
        if self.even:          # one collective (RCCL and gloo alike)
            own = t[self.z0:self.z1].clone()
            _dist.all_gather_into_tensor(t, own, group=self.group)
        else:
            for r, (a, b) in enumerate(self.ranges):
                if b > a:
                    _dist.broadcast(t[a:b], r, group=self.group)
        return t


def member_sharding(model):
    """The ensemble's fit mode: a MemberShard when the job is data-parallel over
    >1 ranks and the ensemble has at least one member per rank (config
    ``dp_mode`` 'auto' | 'members'), else None (batch data parallelism)."""
    mode = getattr(model, 'dp_mode', 'auto')
    if not is_active() or mode == 'batch':
        return None
    if world_size() > model.ensemble_size:
        if mode == 'members':
            raise ValueError(f'dp_mode=members needs ensemble_size >= world size ({world_size()})')
        return None
    return MemberShard(model.ensemble_size)
