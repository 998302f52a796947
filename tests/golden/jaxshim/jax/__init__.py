"""Minimal numpy stand-in for `jax`, used ONLY by tests/golden/gen_golden.py.

jax/jaxlib (pinned 0.4.23 by the reference's requirements.txt) are not installed in this
container and cannot be fetched.  The reference modules call `jax.jit` at import time
(RK.py:174, models.py:92), so this shim provides just enough surface for them to import and run
on numpy in fp64:

* `jit`            -> identity (static_argnums ignored)
* `vmap`           -> python loop over the mapped axis + np.stack
* `lax.fori_loop`  -> python loop
* `numpy`          -> numpy, with `zeros/ones/eye/array/...` returning an ndarray subclass that
                      supports the functional `.at[idx].set(v)` update
* `numpy.linalg.cholesky` -> all-NaN matrix on failure (jax semantics; models.py:250 relies on it)
* `scipy.linalg.solve_triangular` -> scipy's, check_finite=False (NaNs propagate)

It is test infrastructure, never shipped, never imported by the product or on the GPU box.
"""
import numpy as _np

from . import numpy  # noqa: F401  (jax.numpy)
from . import lax  # noqa: F401
from . import scipy  # noqa: F401
from . import config as _config_mod

config = _config_mod.config


def jit(f=None, static_argnums=None, **kw):
    if f is None:
        return lambda g: g
    return f


def vmap(f, in_axes=0, out_axes=0):
    def wrapped(*args):
        axes = in_axes if isinstance(in_axes, (tuple, list)) else (in_axes,) * len(args)
        size = None
        for a, ax in zip(args, axes):
            if ax is not None:
                size = _np.asarray(a).shape[ax]
                break
        outs = []
        for i in range(size):
            call = []
            for a, ax in zip(args, axes):
                if ax is None:
                    call.append(a)
                else:
                    call.append(_np.take(_np.asarray(a), i, axis=ax))
            outs.append(f(*call))
        return _np.stack([_np.asarray(o) for o in outs], axis=out_axes).view(numpy.Array)
    return wrapped
