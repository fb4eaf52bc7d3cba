"""Minimal gym.spaces stand-ins (gym is not a dependency of this engine).

AtariModel (reference envs/atari/model.py:66-67) asserts a Discrete action space and a
Box observation space; real gym spaces are accepted too (duck-typed by ``n`` /
``shape`` + ``dtype``).
"""

import numpy as np


class Discrete(object):
    def __init__(self, n):
        self.n = int(n)
        self.shape = ()
        self.dtype = np.dtype(np.int64)

    def __repr__(self):
        return 'Discrete({})'.format(self.n)

    def __eq__(self, other):
        return isinstance(other, Discrete) and other.n == self.n


class Box(object):
    def __init__(self, low, high, shape=None, dtype=np.float32):
        dtype = np.dtype(dtype)
        if shape is None:
            low = np.asarray(low, dtype)
            shape = low.shape
        self.low = np.broadcast_to(np.asarray(low, dtype), shape).copy()
        self.high = np.broadcast_to(np.asarray(high, dtype), shape).copy()
        self.shape = tuple(shape)
        self.dtype = dtype

    def __repr__(self):
        return 'Box({}, {})'.format(self.shape, self.dtype)

    def __eq__(self, other):
        return isinstance(other, Box) and other.shape == self.shape and other.dtype == self.dtype


def is_discrete(space):
    return hasattr(space, 'n') and not hasattr(space, 'low')


def is_box(space):
    return hasattr(space, 'low') and hasattr(space, 'high') and hasattr(space, 'shape')


def min_scalar_dtype(space):
    """np.min_scalar_type(n) — the actions placeholder dtype (model.py:176-178)."""
    return np.min_scalar_type(space.n)
