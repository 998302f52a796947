"""jax.scipy.linalg stand-in: solve_triangular without finiteness checks (NaNs propagate)."""
import numpy as _np
import scipy.linalg as _sl


def solve_triangular(a, b, lower=False, **kw):
    return _sl.solve_triangular(_np.asarray(a), _np.asarray(b), lower=lower, check_finite=False)
