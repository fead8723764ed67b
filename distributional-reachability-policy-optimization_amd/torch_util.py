"""Small host utilities with the reference's semantics (src/torch_util.py, src/util.py)."""
import random

import numpy as np
import torch
import torch.nn as nn

device = torch.device('cuda' if torch.cuda.is_available() else 'cpu')


def torchify(x, double_to_float=True, int_to_long=True, to_device=True):
    if not torch.is_tensor(x):
        x = torch.from_numpy(x) if isinstance(x, np.ndarray) else torch.tensor(x)
    if x.dtype == torch.double and double_to_float:
        x = x.float()
    elif x.dtype == torch.int and int_to_long:
        x = x.long()
    return x.to(device) if to_device else x


def numpyify(x):
    if isinstance(x, np.ndarray):
        return x
    if torch.is_tensor(x):
        return x.cpu().numpy()
    return np.array(x)


def set_seed(seed):
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    np.random.seed(seed)
    random.seed(seed)


def pythonic_mean(x):
    return sum(x) / len(x)


class Module(nn.Module):
    """nn.Module whose __call__ moves tensor args to the module device (src/torch_util.py:101-113)."""

    def __call__(self, *args, **kwargs):
        args = [x.to(device) if isinstance(x, torch.Tensor) else x for x in args]
        kwargs = {k: v.to(device) if isinstance(v, torch.Tensor) else v for k, v in kwargs.items()}
        return super().__call__(*args, **kwargs)


def freeze_module(module):
    for p in module.parameters():
        p.requires_grad = False
