"""Test-only stand-in for gym 0.17.3 (absent in this image; no network).

Provides just the names the reference's DRPO path touches at import time:
Env, Wrapper, register and the spaces/wrappers/utils submodules. Used ONLY by
tests/golden/make_golden.py in the build container to import the reference.
"""
from . import spaces, wrappers, utils  # noqa: F401


class Env:
    metadata = {}

    def seed(self, seed=None):
        return [seed]


class Wrapper(Env):
    def __init__(self, env):
        self.env = env

    def __getattr__(self, name):
        if name.startswith('_') and name != '_max_episode_steps':
            raise AttributeError(name)
        return getattr(self.env, name)


def register(*args, **kwargs):
    pass
