"""jax.numpy.linalg stand-in: cholesky returns NaNs on failure (jax semantics)."""
import numpy as _np
from numpy.linalg import *  # noqa: F401,F403


def cholesky(a):
    try:
        return _np.linalg.cholesky(a)
    except _np.linalg.LinAlgError:
        out = _np.empty(_np.shape(a))
        out.fill(_np.nan)
        return out
