"""Checkpoint interop with the reference's run directories (src/checkpoint.py:9-96,
main.py:34-71): ``ckpt_{epoch}.pt`` holds ``SMBPO.state_dict()`` (103 keys for
point-robot, including the duplicate ``solver.model_ensemble.*`` copy; ``log_alpha``,
optimizer and scheduler states are not saved, as in the reference) and ``data.pt``
the CheckpointableData metric history.

Loading uses ``torch.load(..., weights_only=True)``: the files hold tensors and
plain Python containers only, so nothing in them is executed."""
from copy import deepcopy
from pathlib import Path

import torch

from .log import default_log as log


class CheckpointableData:
    def __init__(self):
        self._data = {}

    def __getitem__(self, item):
        return self._data[item]

    def append(self, name, value, verbose=False):
        self._data.setdefault(name, []).append(value)
        if verbose:
            log.message(f'{name}: {value:.2f}' if isinstance(value, float) else f'{name}: {value}')

    def state_dict(self):
        return deepcopy(self._data)

    def load_state_dict(self, state_dict):
        self._data = deepcopy(state_dict)

    def __repr__(self):
        return repr(self._data)


def assert_checkpointable(o):
    if isinstance(o, list):
        for x in o:
            assert_checkpointable(x)
    elif isinstance(o, dict):
        for x in o.values():
            assert_checkpointable(x)
    else:
        assert callable(getattr(o, 'state_dict', None)) and callable(getattr(o, 'load_state_dict', None))


class Checkpointer:
    def __init__(self, checkpointable, dir, filename_format):
        assert_checkpointable(checkpointable)
        self.checkpointable = checkpointable
        self.dir = Path(dir)
        self.filename_format = filename_format

    def _path(self, *args):
        return self.dir / self.filename_format.format(*args)

    def save(self, *args):
        c = self.checkpointable
        if isinstance(c, list):
            state = [x.state_dict() for x in c]
        elif isinstance(c, dict):
            state = {k: x.state_dict() for k, x in c.items()}
        else:
            state = c.state_dict()
        torch.save(state, self._path(*args))

    def load(self, *args):
        state = torch.load(self._path(*args), map_location='cpu', weights_only=True)
        c = self.checkpointable
        if isinstance(c, list):
            assert isinstance(state, list)
            for x, sd in zip(c, state):
                x.load_state_dict(sd)
        elif isinstance(c, dict):
            assert isinstance(state, dict)
            for k, x in c.items():
                x.load_state_dict(state[k])
        else:
            c.load_state_dict(state)

    def try_load(self, *args):
        try:
            self.load(*args)
            return True
        except Exception:
            return False

    def load_latest(self, candidates):
        for cand in sorted(candidates, reverse=True):
            if self.try_load(cand):
                return cand
