"""CPU oracle for the full-data GParareal model -- TEST INFRASTRUCTURE, NOT THE PRODUCT.

A numpy/scipy restatement of models.GPjax_p's likelihood and training (models.py:300-417), used
only by tests/ as the checker of nngp_gpfull_lml / nngp_gpfull_fit.  The product path
(nearest-neighbors-gparareal_amd/models.py GPjax_p -> csrc/nngp_gpfull.hip) never imports it.

Parity: pinned against tests/golden/gp_lorenz.npz (tests/golden/gen_golden.py part_gp, produced
by running the reference's GPjax_p on BASELINE configs[0]): the recorded training fan-outs
(theta, fval per fit) and log-likelihood values (tests/test_oracle_golden.py).
"""
import numpy as np
import scipy.linalg
import scipy.optimize
import scipy.spatial.distance

JITTERS = np.arange(-20, -11, dtype=float)   # models.py:378


def gp_kernel(x, y, theta):
    """kernel_np (models.py:300-304): sigma_y^2 * exp(-0.5 * (1/sigma_x^2) * cdist sqeuclidean)."""
    sx, sy = theta
    dist = scipy.spatial.distance.cdist(x, y, metric='sqeuclidean')
    return (sy ** 2) * np.exp(-0.5 * (1 / (sx ** 2)) * dist)


def gp_nlml(x, y, theta, jitter):
    """log_lik -> _log_lik_np -> _fit_gp_np (models.py:306-327); +inf on a failed Cholesky."""
    n = x.shape[0]
    K = gp_kernel(x, x, theta) + np.eye(n) * 10 ** jitter
    try:
        L = np.linalg.cholesky(K)
    except np.linalg.LinAlgError:
        return np.inf
    z = scipy.linalg.solve_triangular(L, y, lower=True)
    alpha = scipy.linalg.solve_triangular(L.T, z, lower=False)
    return -(-0.5 * y.T @ alpha - np.sum(np.log(np.diag(L))) - (n / 2) * np.log(2 * np.pi))


def gp_fit(x, y, theta0, jitter, fatol, xatol):
    """opt_theta (models.py:329-335): scipy Nelder-Mead from theta0."""
    r = scipy.optimize.minimize(lambda th: gp_nlml(x, y, th, jitter), theta0, method='Nelder-Mead',
                                options={'fatol': fatol, 'xatol': xatol})
    return np.asarray(r.x, dtype=float), float(r.fun), int(r.nfev)


def gp_weights(x, y, theta, jitter):
    """_predict's memoised weights (models.py:446-451)."""
    n = x.shape[0]
    L = np.linalg.cholesky(gp_kernel(x, x, theta) + np.eye(n) * 10 ** jitter)
    return np.linalg.solve(L.T, np.linalg.solve(L, y))


def gp_mean(x, alpha, new_x, theta):
    """posterior mean K(x, new_x)^T alpha (models.py:452-453)."""
    return float((gp_kernel(x, np.atleast_2d(new_x), theta).T @ alpha).squeeze())
