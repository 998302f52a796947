"""GPU: the full-data GParareal model (models.GPjax_p -> csrc/nngp_gpfull.hip) against the oracle
(oracle/gpfull.py, pinned to the reference's fixtures) and the reference's own run
(tests/golden/gp_lorenz.npz: Lorenz N=32, BASELINE configs[0]).

Tolerances: the -LML follows the reference's expressions, but the Cholesky's summation order is
the GPU's blocked order, not LAPACK's: single values agree to 1e-9 relative; Nelder-Mead
trajectories that branch on last-bit differences may part, so the fits are compared on the
selected optimum and the run on K / conv_int / iterates (1e-6)."""
import ctypes

import numpy as np
import pytest

import gpfull as GF
from conftest import golden

pytestmark = pytest.mark.gpu


def _dev(torch, a):
    return torch.tensor(np.ascontiguousarray(a, dtype=np.float64), device='cuda')


def _lml(gpu, torch, x, y, coords, jitters, thetas, alpha=False):
    n_pts = len(coords)
    X, Y = _dev(torch, x), _dev(torch, y)
    c = np.ascontiguousarray(coords, dtype=np.int32)
    jx = np.ascontiguousarray(jitters, dtype=float)
    th = np.ascontiguousarray(thetas, dtype=float).reshape(n_pts, 2)
    fv = np.empty(n_pts)
    al = torch.empty((n_pts, x.shape[0]), dtype=torch.float64, device='cuda') if alpha else None
    ip = ctypes.POINTER(ctypes.c_int32)
    dp = ctypes.POINTER(ctypes.c_double)
    gpu._lib.check(gpu.lib().nngp_gpfull_lml(
        X.data_ptr(), x.shape[0], x.shape[1], Y.data_ptr(), n_pts, c.ctypes.data_as(ip), jx.ctypes.data_as(dp),
        th.ctypes.data_as(dp), fv.ctypes.data_as(dp), al.data_ptr() if alpha else None, None))
    torch.cuda.synchronize()
    return fv, (al.cpu().numpy() if alpha else None)


def _tol(x, theta, jit):
    """1e-9 relative, widened by the kernel matrix's condition number (a value at cond ~ 1e20 is
    roundoff-dominated in any summation order, the reference's included)."""
    K = GF.gp_kernel(x, x, theta) + np.eye(x.shape[0]) * 10 ** jit
    with np.errstate(all='ignore'):
        c = np.linalg.cond(K) if np.all(np.isfinite(K)) else np.inf
    return max(1e-9, 1e-14 * c) if np.isfinite(c) else 1e-9


def _close(a, b, rel):
    if np.isinf(b):
        return np.isinf(a) and np.sign(a) == np.sign(b)
    return abs(a - b) <= rel * max(1.0, abs(b))


def test_gpfull_lml_matches_reference_values(gpu):
    import torch
    P = golden('gp_lorenz.npz')
    x, y = P['call1__x'], P['call1__y']
    k = len(P['lml_val'])
    fv, _ = _lml(gpu, torch, x, y, [j % 3 for j in range(k)], P['lml_jitter'], P['lml_theta'])
    for a, b, th, jit in zip(fv, P['lml_val'], P['lml_theta'], P['lml_jitter']):
        assert _close(a, b, _tol(x, th, jit)), (a, b, th, jit)


ORDERS = {'ll64': {'NNGP_GPF_ORDER': '0', 'NNGP_GPF_FMA': '0'}, 'll64_fma': {'NNGP_GPF_ORDER': '0', 'NNGP_GPF_FMA': '1'},
          'rl32': {'NNGP_GPF_ORDER': '1', 'NNGP_GPF_FMA': '0'}}


@pytest.mark.parametrize('order', sorted(ORDERS))
@pytest.mark.parametrize('n', [1, 5, 31, 32, 33, 63, 64, 65, 100, 129, 257, 600])
def test_gpfull_lml_and_weights_vs_oracle(gpu, n, order, monkeypatch):
    """Panel edges (31/32/33 and 63/64/65), several panels, and a 600-row set (the size GParareal
    reaches), in every factor order (NNGP_GPF_ORDER / NNGP_GPF_FMA; each against the oracle, as
    they round differently); a one-matrix slab (NNGP_GPF_SLAB_MB) and the unfused diagonal factor
    (NNGP_GPF_FUSE=0) bitwise the defaults."""
    import torch
    for k, v in ORDERS[order].items():
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(n)
    x = rng.uniform(-1, 1, (n, 3))
    y = np.sin(2 * x) + 0.01 * rng.standard_normal((n, 3))
    thetas = [(0.7, 1.3), (0.2, 0.5), (1.9, 0.05), (0.0, 1.0)]
    jit = [-12.0, -14.0, -11.0, -16.0]
    coords = [0, 1, 2, 0]
    fv, al = _lml(gpu, torch, x, y, coords, jit, thetas, alpha=True)
    monkeypatch.setenv('NNGP_GPF_SLAB_MB', str(max(1, 8 * (n + 1) ** 2 >> 20)))   # one matrix per chunk
    fv1, al1 = _lml(gpu, torch, x, y, coords, jit, thetas, alpha=True)
    assert np.array_equal(fv1, fv) and np.array_equal(np.nan_to_num(al1[:3]), np.nan_to_num(al[:3]))
    if order != 'rl32':   # the diagonal factor in its own launch: bitwise the fused one
        monkeypatch.setenv('NNGP_GPF_FUSE', '0')
        fv2, al2 = _lml(gpu, torch, x, y, coords, jit, thetas, alpha=True)
        assert np.array_equal(fv2, fv) and np.array_equal(np.nan_to_num(al2[:3]), np.nan_to_num(al[:3]))
    # sigma_x = 0: NaN kernel -> failed Cholesky -> +inf (the reference would raise from
    # solve_triangular's finite check here, so there is no reference value to compare with)
    assert np.isinf(fv[3]) and fv[3] > 0
    for i in range(3):
        ref = GF.gp_nlml(x, y[:, coords[i]], np.array(thetas[i]), jit[i])
        assert _close(fv[i], ref, _tol(x, np.array(thetas[i]), jit[i])), (n, i, fv[i], ref)
        if np.isfinite(ref):   # the weights solve K alpha = y backward-stably (alpha itself is
            # as ill-conditioned as K, so it is checked through its residual)
            K = GF.gp_kernel(x, x, np.array(thetas[i])) + np.eye(n) * 10 ** jit[i]
            yy = y[:, coords[i]]
            res = np.abs(K @ al[i] - yy).max()
            assert res <= 1e-12 * (np.abs(K).sum(1).max() * np.abs(al[i]).max() + np.abs(yy).max()), (n, i, res)


def test_gpfull_weights_beyond_the_lds_vector(gpu):
    """More training rows than the alpha solve's LDS vector (7 936): the solve keeps the vector in
    the point's own output row instead -- no row limit, as in the reference's GPjax_p (the rows
    grow by N+1-I per iteration).  A well-conditioned kernel, so the -LML is held to 1e-9 relative
    of the oracle and the weights to a backward-stable residual."""
    import torch
    n = 8200
    rng = np.random.default_rng(8200)
    x = rng.uniform(-1, 1, (n, 2))
    y = np.sin(2 * x) + 0.01 * rng.standard_normal((n, 2))
    theta, jit = (0.3, 0.8), -4.0
    fv, al = _lml(gpu, torch, x, y, [1], [jit], [theta], alpha=True)
    ref = GF.gp_nlml(x, y[:, 1], np.array(theta), jit)
    assert _close(fv[0], ref, 1e-9), (fv[0], ref)
    K = GF.gp_kernel(x, x, np.array(theta)) + np.eye(n) * 10 ** jit
    res = np.abs(K @ al[0] - y[:, 1]).max()
    assert res <= 1e-12 * (np.abs(K).sum(1).max() * np.abs(al[0]).max() + np.abs(y[:, 1]).max()), res


def test_gpfull_fit_matches_reference_fits(gpu):
    """nngp_gpfull_fit on the reference's recorded training fan-outs (models.py:404-407): every
    coordinate's selected optimum (models.py:388-395) matches the reference's."""
    import torch
    from nngp_amd.models import JITTERS, _select_fit
    P = golden('gp_lorenz.npz')
    m = gpu.GPjax_p(n=3, N=32)
    for c in (0, 1):
        x, y, old = P[f'call{c}__x'], P[f'call{c}__y'], P[f'call{c}__old']
        ins, ref = P[f'call{c}__ins'], P[f'call{c}__res']
        m.fatol, m.xatol = P[f'call{c}__tol']
        th, fv, ne = m._fit_batch(_dev(torch, x), _dev(torch, y), [int(i[0]) for i in ins], [i[1] for i in ins],
                                  [old[int(i[0])] for i in ins])
        same = np.mean([_close(a, b, 1e-8) for a, b in zip(fv, ref[:, 2])])
        assert same >= 0.8, f'call{c}: only {same:.0%} of the fits reach the reference fval'
        for j in range(3):
            sl = slice(9 * j, 9 * j + 9)
            g = _select_fit(th[sl], fv[sl], JITTERS)
            r = _select_fit(ref[sl, :2], ref[sl, 2], JITTERS)
            assert g[2] == r[2]
            np.testing.assert_allclose(g[0], r[0], rtol=1e-5, atol=1e-6)
            assert _close(g[1], r[1], 1e-8)


def test_gpfull_predictions_match_oracle(gpu):
    """After fit() on the reference's second training set, the posterior means (the GPU's
    weights and gpf_mean_kernel) equal the oracle's for the model's chosen (theta, jitter)."""
    import torch
    P = golden('gp_lorenz.npz')
    x, y = P['call1__x'], P['call1__y']
    m = gpu.GPjax_p(n=3, N=32)
    m.thetas = [tuple(t) for t in P['call1__old']]
    m.fit(x, y, k=1)
    rng = np.random.default_rng(0)
    for q in x[:5] + 0.01 * rng.standard_normal((5, 3)):
        g = m.predict(q)
        for j in range(3):
            w = GF.gp_weights(x, y[:, j], np.array(m.thetas[j]), m.jitters[j])
            o = GF.gp_mean(x, w, q, np.array(m.thetas[j]))
            assert abs(g[j] - o) <= 1e-7 * max(1.0, abs(o)), (j, g[j], o)


def test_gparareal_lorenz_converges_like_reference(gpu):
    """Parareal(...).run(model='gpjax') on BASELINE configs[0].  Lorenz is chaotic and the
    reference's own Cholesky order is LAPACK's, so K is compared as a band around the reference's
    (like the seed spread of nnGP K); the converged solution must equal the serial
    fine solution (the returned u ends one iterate early, as the reference's does)."""
    P = golden('gp_lorenz.npz')
    F = golden('para_lorenz.npz')['fine']
    ode = gpu.Lorenz(normalization='-11')
    s = gpu.SolverRK(ode.get_vector_field(), Ng=6, Nf=450, F='RK4', G='RK4')
    r = gpu.Parareal(ode, s, [0, 18], 32, epsilon=5e-7, verbose=None).run(model='gpjax')
    print('GParareal K', r['k'], 'reference', int(P['gp__k']), 'conv_int', r['conv_int'],
          'reference', list(P['gp__conv_int']),
          'timings', {k: r['timings'][k] for k in ('F_time', 'G_time', 'mdl_tot_t', 'runtime')})
    assert abs(r['k'] - int(P['gp__k'])) <= 3
    assert r['conv_int'][-1] == 32
    np.testing.assert_allclose(r['u'][:, :, -1], F, rtol=0, atol=1e-3)   # u omits the last iterate


def test_gparareal_fhn_ode_matches_reference_K(gpu):
    """Non-chaotic FHN-ODE (configs.py:7-16: N=40, G=RK2 4/slice, F=RK4 4000/slice): identical
    K and conv_int as the reference's own GParareal run, iterates to 1e-6."""
    P = golden('gp_fhn.npz')
    ode = gpu.FHN_ODE(normalization='-11')
    s = gpu.SolverRK(ode.get_vector_field(), Ng=4, Nf=4000, F='RK4', G='RK2')
    r = gpu.Parareal(ode, s, [0, 40], 40, epsilon=5e-7, verbose=None).run(model='gpjax')
    print('FHN GParareal K', r['k'], 'conv_int', r['conv_int'], 'reference', list(P['gp__conv_int']))
    assert r['k'] == int(P['gp__k'])
    assert r['conv_int'] == [int(c) for c in P['gp__conv_int']]
    np.testing.assert_allclose(r['u'], P['gp__u'], rtol=0, atol=1e-6)


def test_gparareal_checkpoint_resume_is_bitwise(gpu, tmp_path):
    """store_int with model='gpjax': resuming from iteration 2's dump restores the warm-start
    thetas, jitters, hyp and RNG, and reproduces the uninterrupted run exactly."""
    ode = gpu.Lorenz(normalization='-11')
    s = gpu.SolverRK(ode.get_vector_field(), Ng=6, Nf=450, F='RK4', G='RK4')
    full = gpu.Parareal(ode, s, [0, 18], 32, epsilon=5e-7, verbose=None).run(
        model='gpjax', store_int=True, int_dir=str(tmp_path), int_name='gp', early_stop=6)
    p = gpu.Parareal(ode, s, [0, 18], 32, epsilon=5e-7, verbose=None)
    res = p.load_int_dump(str(tmp_path / 'gp' / 'gp_2.npz'), early_stop=6)
    assert res['k'] == full['k'] and res['conv_int'] == full['conv_int']
    assert np.array_equal(np.nan_to_num(res['u'], nan=7.0), np.nan_to_num(full['u'], nan=7.0))


def test_gpfull_fit_chunked_slab_is_bitwise(gpu, monkeypatch):
    """nngp_gpfull_fit with the Nelder-Mead rounds' points factored in several slab chunks
    (NNGP_GPF_SLAB_MB below one round's matrices, as FHN-PDE d_x = 10 at published scale needs)
    returns the same fits, bit for bit, as one slab: chunking only groups independent factors."""
    import torch
    rng = np.random.default_rng(7)
    n, d = 300, 4
    x = rng.uniform(-1, 1, (n, d))
    y = np.sin(2 * x) + 0.01 * rng.standard_normal((n, d))
    m = gpu.GPjax_p(n=d, N=32)
    X, Y = _dev(torch, x), _dev(torch, y)
    coords = [j for j in range(d) for _ in range(9)]
    jit = [float(v) for _ in range(d) for v in range(-20, -11)]
    th0 = [(1.0, 1.0)] * len(coords)
    a = m._fit_batch(X, Y, coords, jit, th0)
    monkeypatch.setenv('NNGP_GPF_SLAB_MB', '3')   # 4 matrices of 301^2 per chunk: 9 chunks per round
    b = m._fit_batch(X, Y, coords, jit, th0)
    for u, v in zip(a, b):
        assert np.array_equal(np.nan_to_num(u, nan=7.0), np.nan_to_num(v, nan=7.0))
