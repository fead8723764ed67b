"""Data parallelism for the hot path.

One process per GPU (torchrun), ``torch.distributed`` over RCCL/xGMI ("nccl") or
gloo for the CPU tests. The path shards with ONE exchange per optimizer step:

  SAC update   each rank draws its own minibatch shard; after the fused backward
               + weight-gradient kernels, the flat gradient of the group being
               stepped (critic+constraint critic 1.37 MB | actor, safe actor and
               log_alpha | multiplier) is mean-all-reduced, then every rank runs
               the identical clip + Adam (clip uses the post-reduce norm).
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


class GradReducer:
    """Mean all-reduce of flat gradient buffers across the data-parallel ranks."""

    def __init__(self, group=None):
        self.group = group
        self.world = world_size()
        self.avg_op = self.world > 1 and _dist.get_backend(group) == 'nccl'

    @property
    def active(self):
        return self.world > 1

    def mean_(self, *tensors):
        if self.world == 1:
            return
        for t in tensors:
            if t is None:
                continue
            if self.avg_op:
                _dist.all_reduce(t, op=_dist.ReduceOp.AVG, group=self.group)
            else:
                _dist.all_reduce(t, group=self.group)
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
                   sol.critic_target_group.data, sol.multiplier.group.data, sol.log_alpha, m.group.data,
                   m.state_normalizer.mean, m.state_normalizer.std, src=src)
    for g in (sol.actor.group, sol.actor_safe.group, sol.critic_group, sol.critic_target_group, sol.multiplier.group,
              m.group):
        g.mark_dirty()
