"""CPU oracle for the nnGParareal hot path -- TEST INFRASTRUCTURE, NOT THE PRODUCT.

Only tests/, __graft_entry__.smoke() and bench.py's `cpu_baseline` leg may import this module,
and only as the checker (or the timed CPU baseline).  The product package
(nearest-neighbors-gparareal_amd/) never imports it and has no CPU fallback.

Two layers:
  * ctypes bindings to oracle/_build/libnngp_oracle.so (oracle/nngp_oracle.c: RHS, RK, -LML,
    Nelder-Mead, kNN, predict -- each citing the reference file:line it restates);
  * `parareal_nngp`, a plain-Python restatement of the reference Parareal loop
    (parareal.py:212-471) and of NNGP_p / BareParareal (models.py:74-226) on top of them.

Parity: pinned against fixtures produced by running the reference itself
(tests/golden/gen_golden.py; see tests/test_oracle_golden.py for the tolerances).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, '_build', 'libnngp_oracle.so')

# enum values mirror include/nngp.h
SYS = {'lorenz': 0, 'hopf': 1, 'tomlab': 2, 'fhn_ode': 3, 'rossler': 4, 'brus': 5,
       'dblpend': 6, 'burgers': 7, 'fhn_pde': 8}
STEP_FIXED, STEP_LINSPACE = 0, 1

# (mn, mx, u0) of the '-11' normalised systems, systems.py:80-288
BOUNDS = {
    'lorenz': ([-17.1, -23, 6], [18.1, 25, 45], [-15, -15, 20]),
    'hopf': ([-23, -23, 0], [23, 23, 1], [0.1, 0.1, -20]),
    'tomlab': ([-12, -12, -12], [12, 12, 12], [4.6722764, 5.2437205e-10, -6.4444208e-10]),
    'fhn_ode': ([-2, -1], [2.1, 1.2], [-1, 1]),
    'rossler': ([-10, -11, 0], [12, 8, 23], [0, -6.78, 0.02]),
    'brus': ([0.4, 0.9], [4, 5], [1, 3.07]),
    'dblpend': ([-2, -2.5, -17, -3.5], [2, 2.5, 1, 3.5], [-0.5, 0, 0, 0]),
}


class CSystem(ctypes.Structure):
    _fields_ = [('kind', ctypes.c_int32), ('d', ctypes.c_int32), ('nx', ctypes.c_int32),
                ('normalized', ctypes.c_int32), ('param', ctypes.c_double * 4),
                ('norm', ctypes.POINTER(ctypes.c_double))]


_lib = None
_dp = ctypes.POINTER(ctypes.c_double)


def build():
    subprocess.run(['make', '-s', '-C', HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        i64, i32, dbl = ctypes.c_int64, ctypes.c_int, ctypes.c_double
        L.orc_rhs.argtypes = [ctypes.POINTER(CSystem), _dp, _dp, _dp]
        L.orc_rk.argtypes = [ctypes.POINTER(CSystem), i32, i32, dbl, dbl, i64, _dp, _dp]
        L.orc_rk_grid.argtypes = [ctypes.POINTER(CSystem), i32, i32, dbl, dbl, i64, i64, i64, _dp, _dp]
        L.orc_rk_batch.argtypes = [ctypes.POINTER(CSystem), i32, i32, i32, _dp, _dp, i64, _dp, _dp, i32]
        L.orc_rk_batch_ex.argtypes = [ctypes.POINTER(CSystem), i32, i32, i32, _dp, _dp, i64, _dp, _dp, i32, i32]
        L.orc_nlml.argtypes = [i32, _dp, _dp, dbl, dbl, dbl]
        L.orc_nlml.restype = dbl
        L.orc_gp_mean_one.argtypes = [i32, _dp, _dp, _dp, dbl, dbl, dbl]
        L.orc_gp_mean_one.restype = dbl
        L.orc_nm_fit.argtypes = [i32, _dp, _dp, _dp, dbl, dbl, dbl, i32, _dp, _dp,
                                 ctypes.POINTER(ctypes.c_int)]
        L.orc_knn.argtypes = [_dp, i64, i32, _dp, i32, ctypes.POINTER(ctypes.c_int32), _dp]
        L.orc_predict.argtypes = [_dp, _dp, i64, i32, _dp, i32, i32, _dp, i32, _dp, dbl, dbl, i32,
                                  _dp, _dp, i32]
        L.orc_d2.argtypes = [_dp, i32, i32, _dp]
        L.orc_max_threads.restype = ctypes.c_int
        L.orc_set_sum_order.argtypes = [i32]
        L.orc_potf2.argtypes = [i32, _dp, _dp]
        L.orc_potf2.restype = i32
        L.orc_solves.argtypes = [i32, _dp, _dp, _dp, _dp]
        L.orc_exp_array.argtypes = [i64, _dp, _dp]
        L.orc_log_array.argtypes = [i64, _dp, _dp]
        for fn in ('nn_exp', 'nn_log', 'nn_pow10', 'nn_sin', 'nn_cos', 'nn_sin_pi'):
            getattr(L, fn).argtypes = [dbl]
            getattr(L, fn).restype = dbl
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(_dp)


def _c(a):
    return np.ascontiguousarray(a, dtype=np.float64)


class System:
    """Oracle-side description of one vector field (+ optional '-11' wrapper)."""

    def __init__(self, name, d=None, nx=0, normalized=True, param=(0.0, 0.0, 0.0, 0.0), mn=None, mx=None,
                 dense=False):
        """dense=True (Burgers, FHN-PDE): rk_batch evaluates the field in the reference's dense
        matrix formulation (systems.py:321-446) -- same results, the reference's cost."""
        self.name = name
        self.dense = bool(dense)
        kind = SYS[name]
        if name in BOUNDS and d is None:
            d = len(BOUNDS[name][0])
        if name == 'burgers':
            nx = d
        if name == 'fhn_pde':
            d = 2 * nx * nx
        self.d = d
        self.normalized = bool(normalized)
        if self.normalized:
            if mn is None:
                mn, mx = BOUNDS[name][0], BOUNDS[name][1]
            mn = np.broadcast_to(np.asarray(mn, dtype=float), (d,))
            mx = np.broadcast_to(np.asarray(mx, dtype=float), (d,))
            w = mx - mn
            self.norm = _c(np.concatenate([mn, w, 2 / (mx - mn)]))
            self.mn, self.mx = mn, mx
        else:
            self.norm = None
        p = (ctypes.c_double * 4)(*list(param) + [0.0] * (4 - len(param)))
        self.c = CSystem(kind, d, nx, int(self.normalized), p,
                         _p(self.norm) if self.norm is not None else ctypes.cast(None, _dp))

    def fit(self, x):
        """Normalize.fit (utils.py:14-19)."""
        if not self.normalized:
            return np.asarray(x, dtype=float)
        return 2 * (np.asarray(x, dtype=float) - self.mn) / (self.mx - self.mn) - 1

    def rhs(self, u):
        u = _c(u)
        out = np.empty(self.d)
        scr = np.empty(self.d)
        lib().orc_rhs(ctypes.byref(self.c), _p(u), _p(out), _p(scr))
        return out

    def rk(self, order, t0, t1, steps, u0, mode=STEP_FIXED):
        u0 = _c(u0)
        out = np.empty(self.d)
        rc = lib().orc_rk(ctypes.byref(self.c), int(order), int(mode), float(t0), float(t1), int(steps), _p(u0), _p(out))
        assert rc == 0
        return out

    def rk_grid(self, order, g0, g1, gsteps, j0, steps, u0):
        u0 = _c(u0)
        out = np.empty(self.d)
        rc = lib().orc_rk_grid(ctypes.byref(self.c), int(order), STEP_LINSPACE, float(g0), float(g1), int(gsteps),
                               int(j0), int(steps), _p(u0), _p(out))
        assert rc == 0
        return out

    def rk_batch(self, order, t0, t1, steps, U0, mode=STEP_FIXED, nthreads=0):
        U0 = _c(U0)
        t0 = _c(t0)
        t1 = _c(t1)
        n = U0.shape[0]
        out = np.empty_like(U0)
        rc = lib().orc_rk_batch_ex(ctypes.byref(self.c), int(order), int(mode), n, _p(t0), _p(t1), int(steps),
                                   _p(U0), _p(out), int(nthreads), int(self.dense))
        assert rc == 0
        return out


def paged(prop, t0, t1, steps, thresh, u0):
    """SolverRK._run_RK_paged (solver.py:86-99) incl. its quirk: every page re-uses the full
    `steps-1` step count over a 1/n_pages sub-interval."""
    if steps > thresh:
        steps = steps - 1
        n_full = int(steps / thresh)
        rem = steps % thresh
        iters = [thresh] * n_full + [rem] * int(rem != 0)
        step = (t1 - t0) / steps
        for temp_steps in iters:
            t1 = t0 + step * temp_steps
            u0 = prop(t0, t1, steps, u0)
            t0 = t1
        return u0
    return prop(t0, t1, steps, u0)


def legacy_paged_batch(system, order, t0, t1, per_slice, thresh, U, nthreads=0):
    """new_lib.RK_last (new_lib.py:57-69) over a batch of slices, on linspace grids: with
    t_steps = per_slice + 1 points above RK_thresh, every page re-uses the full t_steps - 1 point
    count over its sub-interval (float page lengths allowed).  Same float expressions as
    nngp_amd.legacy.LegacySolverRK._rk_last."""
    t0 = np.asarray(t0, dtype=float)
    t1 = np.asarray(t1, dtype=float)
    t_steps = int(per_slice) + 1
    if not t_steps > thresh:
        return system.rk_batch(order, t0, t1, t_steps - 1, U, STEP_LINSPACE, nthreads)
    pts = t_steps - 1
    iters = [thresh] * int(pts / thresh) + [pts % thresh] * (pts % thresh != 0)
    step = (t1 - t0) / pts
    t_s = t0
    for temp in iters:
        t_end = t_s + step * temp
        U = system.rk_batch(order, t_s, t_end, pts - 1, U, STEP_LINSPACE, nthreads)
        t_s = t_end
    return U


def d2_matrix(xm):
    xm = _c(xm)
    m, d = xm.shape
    out = np.empty((m, m))
    lib().orc_d2(_p(xm), m, d, _p(out))
    return out


def nlml(D2, y, theta, jitter_exp):
    D2, y = _c(D2), _c(y)
    return lib().orc_nlml(len(y), _p(D2), _p(y), float(theta[0]), float(theta[1]), float(10.0 ** jitter_exp))


def gp_mean(xm, y, new_x, theta, jitter_exp):
    xm = _c(xm)
    D2 = d2_matrix(xm)
    kd2 = d2_matrix(np.vstack([xm, np.asarray(new_x, dtype=float).reshape(1, -1)]))[-1, :-1].copy()
    return lib().orc_gp_mean_one(len(y), _p(D2), _p(kd2), _p(_c(y)), float(theta[0]), float(theta[1]),
                                 float(10.0 ** jitter_exp))


def nm_fit(D2, y, theta0, jitter_exp, fatol, xatol, maxfev=400):
    D2, y, th0 = _c(D2), _c(y), _c(theta0)
    th = np.empty(2)
    fv = np.empty(1)
    ne = ctypes.c_int(0)
    lib().orc_nm_fit(len(y), _p(D2), _p(y), _p(th0), float(10.0 ** jitter_exp), float(fatol), float(xatol),
                     int(maxfev), _p(th), _p(fv), ctypes.byref(ne))
    return th, float(fv[0]), int(ne.value)


def knn(X, q, m):
    X, q = _c(X), _c(q).reshape(-1)
    idx = np.empty(m, dtype=np.int32)
    dist = np.empty(m)
    lib().orc_knn(_p(X), X.shape[0], X.shape[1], _p(q), int(m), idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), _p(dist))
    return idx, dist


JITTERS = np.arange(-20, -11, dtype=float)   # models.py:186


def predict(X, Y, q, m, theta0, n_restarts=1, fatol=0.1, xatol=0.1, maxfev=400, nthreads=0, return_fits=False):
    X, Y, q, th0 = _c(X), _c(Y), _c(q).reshape(-1), _c(theta0)
    rows, d = X.shape
    nf = d * len(JITTERS) * n_restarts
    assert th0.shape == (nf, 2)
    preds = np.empty(d)
    fits = np.empty((nf, 4))
    jit = _c(JITTERS)
    rc = lib().orc_predict(_p(X), _p(Y), rows, d, _p(q), int(m), len(jit), _p(jit), int(n_restarts), _p(th0),
                           float(fatol), float(xatol), int(maxfev), _p(preds), _p(fits), int(nthreads))
    assert rc == 0
    return (preds, fits) if return_fits else preds


# ---------------------------------------------------------------------------------------------
# Parareal driver restatement (parareal.py:212-471) with the nnGP / Parareal models
# ---------------------------------------------------------------------------------------------
def parareal(system, tspan, N, Ng, Nf, G, F, epsilon=5e-7, model='parareal', nn=10, seed=45,
             n_restarts=1, fatol=0.1, xatol=0.1, u0=None, step_mode=STEP_FIXED, nthreads=0,
             early_stop=None, coarse_grid=False, F_thresh=None, on_iter=None):
    """Returns dict(k, u, err, conv_int, converged, x, D) like Parareal._parareal.  Ng/Nf are
    per-slice step counts; coarse_grid=True takes the legacy initial coarse solution from one
    global grid of N*Ng steps (new_lib.py:902-906) -- with step_mode=STEP_LINSPACE this is the
    legacy new_lib.Parareal loop; F_thresh (with STEP_LINSPACE) adds RK_last's paging of the fine
    solves (new_lib.py:57-69, 940-945).  on_iter(k, state) is called after every iteration
    (progress reports of long runs)."""
    n = system.d
    order = {'RK1': 1, 'RK2': 2, 'RK4': 4, 'RK8': 8}
    oG, oF = order[G], order[F]
    t = np.linspace(tspan[0], tspan[1], num=N + 1)
    u0 = np.asarray(u0, dtype=float)
    rng = np.random.default_rng(seed)                  # models.py:114
    u = np.full((N + 1, n, N + 1), np.nan)
    uG = np.full((N + 1, n, N + 1), np.nan)
    uF = np.full((N + 1, n, N + 1), np.nan)
    err = np.full((N + 1, N), np.nan)
    x = np.zeros((0, n))
    D = np.zeros((0, n))
    conv_int = []
    u[0] = u0[:, None]
    uG[0] = u[0]
    uF[0] = u[0]
    temp = u0
    for i in range(N):                                  # parareal.py:265-270
        if coarse_grid:                                 # new_lib.py:902-906
            temp = system.rk_grid(oG, t[0], t[-1], N * Ng, i * Ng, Ng, temp)
        else:
            temp = system.rk(oG, t[i], t[i + 1], Ng, temp, step_mode)
        uG[i + 1, :, 0] = temp
    u[:, :, 0] = uG[:, :, 0]
    I = 0
    for k in range(N):
        U = u[I:N, :, k]
        if F_thresh is not None:
            assert step_mode == STEP_LINSPACE
            uF[I + 1:N + 1, :, k] = legacy_paged_batch(system, oF, t[I:N], t[I + 1:N + 1], Nf, F_thresh, U, nthreads)
        else:
            uF[I + 1:N + 1, :, k] = system.rk_batch(oF, t[I:N], t[I + 1:N + 1], Nf, U, step_mode, nthreads)
        uG[I + 1, :, k + 1:] = uG[I + 1, :, k].reshape(-1, 1)      # parareal.py:331-333
        uF[I + 1, :, k + 1:] = uF[I + 1, :, k].reshape(-1, 1)
        u[I + 1, :, k + 1:] = uF[I + 1, :, k].reshape(-1, 1)
        I = I + 1
        x = np.vstack([x, u[I - 1:N, :, k]])                          # :336-337
        D = np.vstack([D, uF[I:N + 1, :, k] - uG[I:N + 1, :, k]])
        if I == N:                                                   # :343-348
            err[:, k] = np.linalg.norm(u[:, :, k + 1] - u[:, :, k], np.inf, 1)
            err[-1, k] = np.nextafter(epsilon, 0)
            break
        for i in range(I, N):                                        # :359-382
            uG[i + 1, :, k + 1] = system.rk(oG, t[i], t[i + 1], Ng, u[i, :, k + 1], step_mode)
            if model == 'parareal':
                preds = uF[i + 1, :, k] - uG[i + 1, :, k]           # models.py:82-83
            else:
                m = max(10, k + 2) if nn == 'adaptive' else nn      # models.py:172-175
                m = min(m, x.shape[0])            # argsort(...)[:nn] keeps every row if fewer
                nf = n * len(JITTERS) * n_restarts
                th0 = rng.integers(-8, 0, (nf, 2)).astype(float)    # models.py:192 (same stream)
                preds = predict(x, D, u[i, :, k + 1], m, th0, n_restarts, fatol, xatol, nthreads=nthreads)
            u[i + 1, :, k + 1] = preds + uG[i + 1, :, k + 1]
        if np.any(np.isnan(uG[:, :, k + 1])):
            raise Exception('NaN values in initial coarse solve - increase Ng!')
        err[:, k] = np.linalg.norm(u[:, :, k + 1] - u[:, :, k], np.inf, 1)   # :402-403
        err[I, k] = 0
        II = I
        for p in range(II + 1, N + 1):                                # :408-416
            if err[p, k] < epsilon:
                u[p, :, k + 2:] = u[p, :, k + 1].reshape(-1, 1)
                uG[p, :, k + 2:] = uG[p, :, k + 1].reshape(-1, 1)
                uF[p, :, k + 1:] = uF[p, :, k].reshape(-1, 1)
                I = I + 1
            else:
                break
        conv_int.append(I)
        if on_iter is not None:
            on_iter(k, {'I': I, 'u': u[:, :, :k + 2], 'err': err[:, :k + 1]})
        if I == N:
            break
        if early_stop is not None and k == early_stop - 1:
            break
    return {'t': t, 'u': u[:, :, :k + 1], 'err': err[:, :k + 1], 'k': k + 1, 'x': x, 'D': D,
            'converged': I == N, 'conv_int': conv_int}
