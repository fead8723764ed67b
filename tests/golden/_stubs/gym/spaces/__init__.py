import numpy as np


class Space:
    def seed(self, seed=None):
        return [seed]


class Box(Space):
    def __init__(self, low, high, shape=None, dtype=np.float32):
        if shape is None:
            shape = np.shape(low)
        self.shape = tuple(shape)
        self.low = np.broadcast_to(np.asarray(low, dtype=dtype), self.shape).copy()
        self.high = np.broadcast_to(np.asarray(high, dtype=dtype), self.shape).copy()
        self.dtype = dtype


class Discrete(Space):
    def __init__(self, n):
        self.n = n
        self.shape = ()
