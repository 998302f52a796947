"""jax.numpy stand-in: numpy plus a functional `.at[].set()` on arrays (see jax/__init__.py)."""
import numpy as _np
from numpy import *  # noqa: F401,F403
from numpy import pi, inf, nan  # noqa: F401

from . import _linalg as linalg  # noqa: F401


class _AtIndexer:
    def __init__(self, arr):
        self._arr = arr

    def __getitem__(self, idx):
        arr = self._arr

        class _Setter:
            def set(self_inner, val):
                out = _np.array(arr, copy=True).view(Array)
                out[idx] = val
                return out

            def add(self_inner, val):
                out = _np.array(arr, copy=True).view(Array)
                out[idx] += val
                return out
        return _Setter()


class Array(_np.ndarray):
    @property
    def at(self):
        return _AtIndexer(self)


def _wrap(fn):
    def inner(*a, **k):
        return _np.asarray(fn(*a, **k)).view(Array)
    inner.__name__ = fn.__name__
    return inner


zeros = _wrap(_np.zeros)
ones = _wrap(_np.ones)
eye = _wrap(_np.eye)
empty = _wrap(_np.empty)
full = _wrap(_np.full)
array = _wrap(_np.array)
asarray = _wrap(_np.asarray)
hstack = _wrap(_np.hstack)
vstack = _wrap(_np.vstack)
concatenate = _wrap(_np.concatenate)
zeros_like = _wrap(_np.zeros_like)
