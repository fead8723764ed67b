"""HBM-resident circular replay buffers (src/sampling.py:12-151, 215-251).

Same component order and semantics as the reference (COMPONENT_NAMES is
positional: SMBPO indexes REWARD=3 and CONSTRAINT_VALUE=6). The write pointer
lives on the device (``_pointer``, like the reference's registered buffer) so
that device kernels (the fused rollout) can append without a host round trip;
a host mirror avoids device->host syncs whenever the host knows the value.
"""
import torch
import torch.nn as nn

from .torch_util import device as default_device


def sample_without_replacement(high, size, device):
    """``random_indices(high, size, replace=False)`` (src/torch_util.py:41-44) on the
    device: a keyed pseudo-random permutation evaluated at 0..size-1
    (drpo_sample_without_replacement). The key comes from torch's host generator,
    so ``torch.manual_seed`` makes it reproducible; no host<->device sync."""
    from . import _lib
    if not 0 <= size <= high:
        raise ValueError(f'cannot take {size} distinct indices out of {high}')
    idx = torch.empty(size, dtype=torch.int64, device=device)
    seed, ctr = (int(v) for v in torch.randint(0, 2 ** 62, (2,)))
    _lib.check(_lib.lib().drpo_sample_without_replacement(_lib.ptr(idx), size, high, seed, ctr, _lib.stream()),
               'sample_without_replacement')
    return idx


class SampleBuffer(nn.Module):
    COMPONENT_NAMES = ('states', 'actions', 'next_states', 'rewards', 'dones')

    def __init__(self, state_dim, action_dim, capacity, discrete_actions=False, device=default_device):
        super().__init__()
        self.state_dim = state_dim
        self.action_dim = action_dim
        self.capacity = capacity
        self.discrete_actions = discrete_actions
        self.device = device
        self._bufs = {}
        self.register_buffer('_pointer', torch.tensor(0, dtype=torch.long, device=device))
        self._host_ptr = 0            # None when only the device value is current
        if discrete_actions:
            assert action_dim == 1
            adt, ash = torch.int, []
        else:
            adt, ash = torch.float, [action_dim]
        for name, dt, shape in (('states', torch.float, [state_dim]), ('actions', adt, ash),
                                ('next_states', torch.float, [state_dim]), ('rewards', torch.float, []),
                                ('dones', torch.bool, [])):
            self._create_buffer(name, dt, shape)

    def _create_buffer(self, name, dtype, shape):
        assert name not in self._bufs
        buf = torch.zeros(self.capacity, *shape, dtype=dtype, device=self.device)
        self.register_buffer('_' + name, buf)
        self._bufs[name] = buf

    # ---- pointer ---------------------------------------------------------
    @property
    def pointer(self):
        if self._host_ptr is None:
            self._host_ptr = int(self._pointer.item())
        return self._host_ptr

    def _device_advanced(self):
        """A device kernel moved _pointer; the host mirror is stale until read."""
        self._host_ptr = None

    def _set_pointer(self, p):
        self._host_ptr = int(p)
        self._pointer.fill_(int(p))

    def __len__(self):
        return min(self.pointer, self.capacity)

    def load_state_dict(self, state_dict, strict=True):
        r = super().load_state_dict(state_dict, strict)
        self._host_ptr = None
        return r

    @classmethod
    def from_state_dict(cls, state_dict, device=default_device):
        assert set(state_dict.keys()) == {*(f'_{n}' for n in cls.COMPONENT_NAMES), '_pointer'}
        states, actions = state_dict['_states'], state_dict['_actions']
        for n in cls.COMPONENT_NAMES:
            assert len(state_dict[f'_{n}']) == len(states)
        buf = cls(state_dim=states.shape[1], action_dim=actions.shape[1], capacity=len(states),
                  discrete_actions=not actions.dtype.is_floating_point, device=device)
        buf.load_state_dict(state_dict)
        return buf

    # ---- host-side access (src/sampling.py:97-151) -------------------------
    def _get1(self, name):
        buf = self._bufs[name]
        p = self.pointer
        if p <= self.capacity:
            return buf[:p]
        i = p % self.capacity
        return torch.cat([buf[i:], buf[:i]])

    def get(self, *names, device=default_device, as_dict=False):
        if len(names) == 0:
            names = self.COMPONENT_NAMES
        bufs = [self._get1(n).to(device) for n in names]
        if as_dict:
            return dict(zip(names, bufs))
        return bufs if len(bufs) > 1 else bufs[0]

    def append(self, **kwargs):
        assert set(kwargs.keys()) == set(self.COMPONENT_NAMES)
        p = self.pointer
        i = p % self.capacity
        for n in self.COMPONENT_NAMES:
            self._bufs[n][i] = torch.as_tensor(kwargs[n], device=self.device)
        self._set_pointer(p + 1)

    def extend(self, **kwargs):
        assert set(kwargs.keys()) == set(self.COMPONENT_NAMES)
        n = len(list(kwargs.values())[0])
        assert n <= self.capacity, 'We do not support extending by more than buffer capacity'
        p = self.pointer
        i = p % self.capacity
        end = i + n
        for name in self.COMPONENT_NAMES:
            buf, arg = self._bufs[name], torch.as_tensor(kwargs[name]).to(self.device)
            if end <= self.capacity:
                buf[i:end] = arg
            else:
                fit = self.capacity - i
                buf[-fit:] = arg[:fit]
                buf[:end - self.capacity] = arg[-(end - self.capacity):]
        self._set_pointer(p + n)

    def sample(self, batch_size, replace=True, device=default_device, include_indices=False):
        if replace:
            idx = torch.randint(len(self), [batch_size], device=self.device)
        else:
            idx = sample_without_replacement(len(self), batch_size, self.device)
        bufs = [self._bufs[n][idx].to(device) for n in self.COMPONENT_NAMES]
        return (bufs, idx) if include_indices else bufs


class SafetySampleBuffer(SampleBuffer):
    COMPONENT_NAMES = (*SampleBuffer.COMPONENT_NAMES, 'violations')

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self._create_buffer('violations', torch.bool, [])


class ConstraintSafetySampleBuffer(SafetySampleBuffer):
    COMPONENT_NAMES = (*SafetySampleBuffer.COMPONENT_NAMES, 'constraint_values')

    def __init__(self, *args, **kwargs):
        con_dim = kwargs.pop('con_dim')
        super().__init__(*args, **kwargs)
        self.con_dim = con_dim
        self._create_buffer('constraint_values', torch.float, [] if con_dim == 1 else [con_dim])


class DummyModuleWrapper:
    """Keeps a module out of its parent's state_dict (src/torch_util.py:116-133)."""

    def __init__(self, module):
        assert isinstance(module, nn.Module)
        self.__dict__['_module'] = module

    def __getattr__(self, attr):
        if attr == '_module':
            return self.__dict__['_module']
        return getattr(self._module, attr)

    def __setattr__(self, attr, value):
        setattr(self.__dict__['_module'], attr, value)

    def __len__(self):
        return len(self._module)
