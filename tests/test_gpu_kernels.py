"""GPU parity of every C-ABI entry point against the CPU oracle (oracle/) and the reference's own
fixtures (tests/golden/).  Marked `gpu`; run on an MI355X with `pytest -m gpu`.

Tolerances: the kernels evaluate the same operations in the same order as the oracle
(-ffp-contract=off on both sides; exp/log/10^x/sin/cos are the repo's own fully specified
routines, csrc/nngp_math.h == oracle), so right-hand sides, whole RK trajectories and GP fits
are bit-exact GPU vs oracle.  Against the reference's own fixtures: bit-exact for polynomial
ODEs, 1e-12 relative for PDE rows (BLAS summation order) and sin/cos fields (libm ulps)."""
import ctypes

import numpy as np
import pytest

import oracle as O
from conftest import golden
from systems_table import EXACT, KEYS, RK_KEYS, TRIG, oracle_system, product_ode  # noqa: F401

pytestmark = pytest.mark.gpu


def _t(torch, a, dtype=None):
    return torch.tensor(np.ascontiguousarray(a), dtype=dtype or torch.float64, device='cuda')


@pytest.mark.parametrize('key', KEYS)
def test_rhs_kernel_vs_oracle_and_reference(gpu, key):
    R = golden('rhs.npz')
    ode = product_ode(gpu, key)
    f = ode.get_vector_field()
    U = R[key + '__u']
    got = f(0.0, U)
    ora = np.array([oracle_system(key).rhs(u) for u in U])
    assert np.array_equal(got, ora)        # incl. sin/cos: the shared fully specified routines
    ref = R[key + '__f']
    tol = 0 if key in EXACT else 1e-12 * max(1.0, np.max(np.abs(ref)))
    assert np.max(np.abs(got - ref)) <= tol


@pytest.mark.parametrize('key', RK_KEYS)
@pytest.mark.parametrize('tab', ['RK1', 'RK2', 'RK4', 'RK8'])
@pytest.mark.parametrize('mode', ['fixed', 'linspace'])
def test_rk_batch_vs_oracle(gpu, key, tab, mode):
    import torch
    R = golden('rk.npz')
    k = f'{key}__{tab}'
    u0 = R[k + '__u0']
    t0, t1, steps = R[k + '__span']
    ode = product_ode(gpu, key)
    s = gpu.SolverRK(ode.get_vector_field(), Ng=int(steps), Nf=int(steps), F=tab, G=tab, step_mode=mode)
    # a batch of 5 slices with different initial values and spans
    rng = np.random.default_rng(3)
    U0 = u0[None, :] + 1e-3 * rng.standard_normal((5, len(u0)))
    T0 = t0 + np.arange(5) * (t1 - t0)
    T1 = T0 + (t1 - t0)
    out = s.run_F_batch(_t(torch, T0), _t(torch, T1), _t(torch, U0)).cpu().numpy()
    so = oracle_system(key)
    m = O.STEP_FIXED if mode == 'fixed' else O.STEP_LINSPACE
    ora = np.array([so.rk(int(tab[2:]), T0[i], T1[i], int(steps), U0[i], m) for i in range(5)])
    assert np.array_equal(out, ora)
    # slice 0 is exactly the reference fixture's input
    one = s.run_F_batch(_t(torch, [t0]), _t(torch, [t1]), _t(torch, u0[None, :])).cpu().numpy()[0]
    ref = R[k + ('__fixed' if mode == 'fixed' else '__linspace')]
    tol = 0 if key in EXACT else (1e-12 if key in TRIG else 1e-13) * max(1.0, np.max(np.abs(ref)))
    assert np.max(np.abs(one - ref)) <= tol


@pytest.mark.parametrize('key', ['lorenz', 'lorenz_id', 'hopf', 'tomlab', 'rossler', 'fhn_ode', 'brus', 'dblpend'])
@pytest.mark.parametrize('n', [1, 5, 37, 300, 5000])
def test_rk_group_kernel_equals_lane_kernel(gpu, key, n, monkeypatch):
    """The lane-group kernel (one slice per 4- or 16-lane group, components across lanes) is
    bitwise the one-lane-per-slice kernel, for partial and full waves and past its size limit
    (n=5000 at 16 lanes per slice falls back to the lane kernel); d = 2, 3 and 4."""
    import torch
    ode = product_ode(gpu, key)
    s = gpu.SolverRK(ode.get_vector_field(), Ng=7, Nf=200, F='RK4', G='RK4')
    rng = np.random.default_rng(n)
    lo, hi = (-0.9, 0.9) if key != 'lorenz_id' else (-15.0, 15.0)
    U0 = rng.uniform(lo, hi, (n, len(ode.get_init_cond())))
    T0 = rng.uniform(0, 1, n)
    T1 = T0 + 0.5
    args = (_t(torch, T0), _t(torch, T1), _t(torch, U0))
    monkeypatch.setenv('NNGP_RK_GROUP', '1')
    grp = s.run_F_batch(*args).cpu().numpy()
    monkeypatch.setenv('NNGP_RK_GROUP', '0')
    lane = s.run_F_batch(*args).cpu().numpy()
    assert np.array_equal(grp, lane, equal_nan=True)
    assert np.all(np.isfinite(grp))


@pytest.mark.parametrize('nx', [10, 20])
def test_field_kernel_thread_overrides(gpu, nx, monkeypatch):
    """Every valid NNGP_RK_THREADS layout of the field kernel is bitwise the default one; a block
    larger than the chosen variant's launch bound is refused with an error, not launched."""
    import torch
    ode = gpu.FHN_PDE(d_x=nx)
    d = 2 * nx * nx
    s = gpu.SolverRK(ode.get_vector_field(), Ng=1, Nf=20, F='RK8', G='RK1')
    rng = np.random.default_rng(nx)
    U0 = _t(torch, np.clip(ode.get_init_cond()[None, :] + 0.01 * rng.standard_normal((6, d)), -1, 1))
    T0 = _t(torch, np.arange(6) * 0.5)
    T1 = T0 + 0.5
    ref = s.run_F_batch(T0, T1, U0).cpu().numpy()
    for thr in (64, 128, 192, 256, 384, 512, 832, 1024):
        ept = -(-d // thr)
        ok = ept <= 8 and thr <= (1024 if ept <= 1 else 512 if ept <= 2 else 256)
        monkeypatch.setenv('NNGP_RK_THREADS', str(thr))
        if ok:
            assert np.array_equal(s.run_F_batch(T0, T1, U0).cpu().numpy(), ref), thr
        else:
            with pytest.raises(gpu.NNGPError):
                s.run_F_batch(T0, T1, U0)


@pytest.mark.parametrize('nx,norm,mode', [(4, None, 'fixed'), (10, '-11', 'linspace'), (16, None, 'fixed'),
                                          (20, None, 'linspace'), (20, '-11', 'fixed'), (32, None, 'fixed')])
def test_fhn_point_pair_kernel_equals_element_kernel(gpu, nx, norm, mode, monkeypatch):
    """FHN-PDE's point-pair field kernel (one thread per grid point: u and v of the point, the
    reaction terms' own/partner values from registers; the default from 16x16 points) is bitwise
    the element-per-thread kernel (NNGP_FHN_PAIR=0) and the oracle, fixed and linspace grids, RK4
    and RK8, up to d = 2048 (below 16x16 both runs take the element kernel)."""
    import torch
    ode = gpu.FHN_PDE(d_x=nx, normalization=norm) if norm else gpu.FHN_PDE(d_x=nx)
    d = 2 * nx * nx
    rng = np.random.default_rng(nx)
    n = 5
    U0 = np.clip(ode.get_init_cond()[None, :] + 0.01 * rng.standard_normal((n, d)), -1, 1)
    T0 = np.arange(n) * 0.05
    T1 = T0 + 0.05   # inside the explicit stability limit of the finest grid's diffusion
    for tab in ('RK4', 'RK8'):
        s = gpu.SolverRK(ode.get_vector_field(), Ng=1, Nf=12, F=tab, G='RK1', step_mode=mode)
        monkeypatch.delenv('NNGP_FHN_PAIR', raising=False)
        pair = s.run_F_batch(_t(torch, T0), _t(torch, T1), _t(torch, U0)).cpu().numpy()
        monkeypatch.setenv('NNGP_FHN_PAIR', '0')
        elem = s.run_F_batch(_t(torch, T0), _t(torch, T1), _t(torch, U0)).cpu().numpy()
        assert np.all(np.isfinite(pair)) and np.array_equal(pair, elem), (nx, tab)
        so = O.System('fhn_pde', nx=nx, mn=-1, mx=1) if norm else O.System('fhn_pde', nx=nx, normalized=False)
        m = O.STEP_FIXED if mode == 'fixed' else O.STEP_LINSPACE
        ora = np.array([so.rk(int(tab[2:]), T0[i], T1[i], 12, U0[i], m) for i in range(n)])
        assert np.array_equal(pair, ora), (nx, tab)


def test_rk_batch_uF_may_alias_u0(gpu):
    import torch
    ode = gpu.Burgers(d_x=128, normalization='-11')
    s = gpu.SolverRK(ode.get_vector_field(), 4, 50, 'RK8', 'RK1')
    U = _t(torch, np.tile(ode.get_init_cond(), (3, 1)))
    ref = s.run_F_batch(_t(torch, [0.0] * 3), _t(torch, [0.04] * 3), U.clone()).cpu().numpy()
    s.run_F_batch(_t(torch, [0.0] * 3), _t(torch, [0.04] * 3), U, out=U)
    assert np.array_equal(U.cpu().numpy(), ref)


@pytest.mark.parametrize('tag', ['paged', 'paged73'])
def test_paged_solver_matches_reference(gpu, tag):
    R = golden('rk.npz')
    t0, t1, steps, thresh = R[tag + '__lorenz__args']
    ode = gpu.Lorenz(normalization='-11')
    s = gpu.SolverRK(ode.get_vector_field(), Ng=6, Nf=int(steps), F='RK4', G='RK4',
                     thresh=thresh if tag == 'paged73' else int(thresh))
    out = s.run_F(t0, t1, R['paged__lorenz__u0'])
    assert np.array_equal(out, R[tag + '__lorenz__out'])


def test_rk_batch_grid_vs_oracle(gpu):
    import torch
    ode = gpu.Hopf(normalization='-11')
    cs = ode.get_vector_field().csystem(torch.device('cuda'))
    so = oracle_system('hopf')
    u0 = np.array([0.1, 0.2, -0.99])
    n, per = 8, 16
    U = torch.empty((n + 1, 3), dtype=torch.float64, device='cuda')
    U[0] = _t(torch, u0)
    L = gpu.lib()
    g0 = _t(torch, [-20.0])
    g1 = _t(torch, [-19.0])
    for i in range(n):
        j0 = torch.tensor([i * per], dtype=torch.int64, device='cuda')
        gpu._lib.check(L.nngp_rk_batch_grid(ctypes.byref(cs), 1, 1, g0.data_ptr(), g1.data_ptr(), n * per,
                                            j0.data_ptr(), per, U[i:i + 1].data_ptr(), U[i + 1:i + 2].data_ptr(), None))
    x = u0
    for i in range(n):
        x = so.rk_grid(1, -20.0, -19.0, n * per, i * per, per, x)
    assert np.array_equal(U[-1].cpu().numpy(), x)


def test_parareal_update_kernel(gpu):
    import torch
    rng = np.random.default_rng(1)
    a, b, c = (rng.standard_normal(1000) for _ in range(3))
    A, B, C = (_t(torch, v) for v in (a, b, c))
    out = torch.empty_like(A)
    gpu._lib.check(gpu.lib().nngp_parareal_update(1000, A.data_ptr(), B.data_ptr(), C.data_ptr(), out.data_ptr(), None))
    assert np.array_equal(out.cpu().numpy(), (a - b) + c)
    gpu._lib.check(gpu.lib().nngp_parareal_update(1000, A.data_ptr(), B.data_ptr(), None, out.data_ptr(), None))
    assert np.array_equal(out.cpu().numpy(), a - b)


# ---------------------------------------------------------------------------------- GP pieces
@pytest.mark.parametrize('rows,d,m', [(640, 3, 10), (3000, 128, 15), (700, 200, 20), (33, 3, 33), (5000, 2, 12),
                                     (1100, 128, 15), (2000, 128, 64), (90, 5, 48)])
def test_knn_vs_oracle(gpu, rows, d, m):
    import torch
    rng = np.random.default_rng(rows + d)
    X = rng.standard_normal((rows, d))
    X[5] = X[rows // 2]                          # exact duplicate -> tie broken by index
    q = X[rows // 2] + 1e-3
    idx = torch.empty(m, dtype=torch.int32, device='cuda')
    dist = torch.empty(m, dtype=torch.float64, device='cuda')
    Xt, qt = _t(torch, X), _t(torch, q)
    gpu._lib.check(gpu.lib().nngp_knn(Xt.data_ptr(), rows, d, qt.data_ptr(), m, idx.data_ptr(), dist.data_ptr(), None))
    oi, od = O.knn(X, q, m)
    assert np.array_equal(idx.cpu().numpy(), oi)
    assert np.array_equal(dist.cpu().numpy(), od)


@pytest.mark.parametrize('key_lds', ['0', '1'])
@pytest.mark.parametrize('rows,d,m,dups', [(30000, 3, 18, 0), (20000, 3, 64, 0), (9000, 3, 18, 400),
                                          (4097, 2, 12, 0), (14336, 3, 18, 0), (14337, 3, 18, 0),
                                          (6000, 3, 64, 300)])
def test_knn_streaming_select_vs_oracle(gpu, rows, d, m, dups, key_lds, monkeypatch):
    """rows > 4 096: the select streams its keys from memory through the radix threshold passes
    (NNGP_KEY_LDS=1, the default: up to 14 336 rows from a copy staged once in LDS); with `dups`
    copies of the query's nearest row more than SEL_CAND (256) rows tie at the threshold and the m
    rounds take over.  Bitwise the oracle either way (ordered by distance, then row)."""
    import torch
    monkeypatch.setenv('NNGP_KEY_LDS', key_lds)
    rng = np.random.default_rng(rows + d + dups)
    X = rng.standard_normal((rows, d))
    q = X[rows // 3] + 1e-3
    if dups:
        X[rng.choice(rows, size=dups, replace=False)] = X[rows // 3]
    idx = torch.empty(m, dtype=torch.int32, device='cuda')
    dist = torch.empty(m, dtype=torch.float64, device='cuda')
    Xt, qt = _t(torch, X), _t(torch, q)
    gpu._lib.check(gpu.lib().nngp_knn(Xt.data_ptr(), rows, d, qt.data_ptr(), m, idx.data_ptr(), dist.data_ptr(), None))
    oi, od = O.knn(X, q, m)
    assert np.array_equal(idx.cpu().numpy(), oi)
    assert np.array_equal(dist.cpu().numpy(), od)


def _nm_case(m, d, seed):
    rng = np.random.default_rng(seed)
    base = rng.uniform(-0.5, 0.5, size=d)
    xm = base + 0.05 * rng.standard_normal((m, d))
    ym = 0.01 * np.sin(3 * xm) + 1e-5 * rng.standard_normal((m, d))
    return xm, ym


@pytest.mark.parametrize('m,d,tol', [(10, 3, 0.1), (15, 3, 1e-3), (18, 3, 0.1), (30, 3, 0.1), (15, 128, 0.1)])
def test_nm_fit_batch_vs_oracle(gpu, m, d, tol):
    mdl = gpu.NNGP_p(n=d, N=4, fatol=tol, xatol=tol, seed=7)
    xm, ym = _nm_case(m, d, m * 100 + d)
    coords = [c for c in range(min(d, 8)) for _ in range(9)]
    jidx = [j for _ in range(min(d, 8)) for j in range(9)]
    th0 = mdl.draw_thetas(1)[:len(coords)]
    res = mdl.fit_batch(xm, ym, coords, jidx, th0)
    D2 = O.d2_matrix(xm)
    exact = 0
    for f in range(len(coords)):
        th, fv, ne = O.nm_fit(D2, ym[:, coords[f]], th0[f], gpu.models.JITTERS[jidx[f]], tol, tol)
        same = ne == res['nfev'][f] and np.array_equal(th, res['theta'][f]) and fv == res['fval'][f]
        exact += same
        if not same:   # an ulp in exp/log/pow may redirect NM; the optimum value must still agree
            assert abs(fv - res['fval'][f]) <= 1e-6 * max(1.0, abs(fv)) or np.isinf(fv) == np.isinf(res['fval'][f])
    assert exact == len(coords)   # shared exp/log/10^x: bitwise


@pytest.mark.parametrize('lpf', ['4', '1'])
@pytest.mark.parametrize('m,d,dup', [(10, 3, False), (15, 3, True), (15, 128, False), (15, 128, True)])
def test_nm_lanes_kernel_vs_oracle(gpu, m, d, dup, lpf, monkeypatch):
    """The throughput fits kernel (csrc/nngp_nmlane.hip: 4 lanes per fit, exact m, work queue;
    forced by NNGP_NM_LANES=1) through nngp_nm_fit_batch: every fit -- theta, -LML and nfev -- bit
    for bit the oracle's Nelder-Mead (oracle/nngp_oracle.c orc_nm_fit).  d = 128: all 1 152
    (coordinate, jitter) fits of a Burgers-sized prediction; dup: two neighbours coincide, so the
    low-jitter kernels are singular and their Cholesky fails (NaN -> +inf) on the way."""
    monkeypatch.setenv('NNGP_NM_LANES', '1')
    monkeypatch.setenv('NNGP_NM_LPF', lpf)   # 4 lanes per fit, or one fit per lane
    mdl = gpu.NNGP_p(n=d, N=4, fatol=0.1, xatol=0.1, seed=7)
    xm, ym = _nm_case(m, d, m * 100 + d + 1)
    if dup:
        xm[m - 1] = xm[1]
    coords = [c for c in range(d) for _ in range(9)]
    jidx = [j for _ in range(d) for j in range(9)]
    th0 = mdl.draw_thetas(1)[:len(coords)]
    res = mdl.fit_batch(xm, ym, coords, jidx, th0)
    D2 = O.d2_matrix(xm)
    bad = []
    for f in range(len(coords)):
        th, fv, ne = O.nm_fit(D2, ym[:, coords[f]], th0[f], gpu.models.JITTERS[jidx[f]], 0.1, 0.1)
        if not (ne == res['nfev'][f] and np.array_equal(th, res['theta'][f]) and
                (fv == res['fval'][f] or (np.isnan(fv) and np.isnan(res['fval'][f])))):
            bad.append((f, ne, res['nfev'][f], fv, res['fval'][f]))
    assert not bad, bad[:5]


def test_gp_mean_vs_oracle(gpu):
    L = golden('lml.npz')
    mdl = gpu.NNGP_p(n=3, N=4)
    th = L['thetas'][40:43]
    got = mdl.gp_mean(L['xm'], L['ym'], L['new_x'], th, np.array([5, 5, 5], dtype=np.int32))
    for j in range(3):
        ora = O.gp_mean(L['xm'], L['ym'][:, j], L['new_x'], th[j], -15.0)
        assert got[j] == ora                                   # same operation order: bitwise
        ref = L['post_mean_jit15'][40 + j, j]
        assert abs(got[j] - ref) <= 1e-8


def test_predict_d128_vs_oracle_and_reference(gpu):
    import torch
    P = golden('preds_d128.npz')
    mdl = gpu.NNGP_p(n=128, N=4, nn=15, seed=45)
    X, Y = _t(torch, P['X']), _t(torch, P['Y'])
    th0 = mdl.draw_thetas(1)
    assert np.array_equal(th0, P['rnd'])
    fits = torch.empty((1152, 4), dtype=torch.float64, device='cuda')
    preds = mdl.predict_device(X, Y, X.shape[0], _t(torch, P['new_x'].reshape(-1)), _t(torch, th0),
                               fits_out=fits).cpu().numpy()
    ora, ofits = O.predict(P['X'], P['Y'], P['new_x'], 15, th0, return_fits=True)
    f = fits.cpu().numpy()
    assert np.array_equal(f, ofits)
    assert np.max(np.abs(preds - ora)) <= 1e-12 * np.max(np.abs(ora))
    sc = np.max(np.abs(P['preds']))
    assert (np.abs(preds - P['preds']) <= 1e-8 * sc).mean() >= 0.97
    assert np.max(np.abs(preds - P['preds'])) <= 5e-2 * sc


def test_fused_predict_equals_unfused_get_preds(gpu):
    import torch
    xm, ym = _nm_case(12, 5, 9)
    X = np.vstack([xm, xm + 0.3])
    Y = np.vstack([ym, ym * 0.5])
    q = xm[3] + 0.01
    a = gpu.NNGP_p(n=5, N=4, nn=12, seed=11)
    b = gpu.NNGP_p(n=5, N=4, nn=12, seed=11)
    a.fit(X, Y, k=0)
    fused = a.predict(q.reshape(1, -1), None, None, i=0)
    idx, _ = O.knn(X, q, 12)
    unfused = b.get_preds(X[idx], Y[idx], 5, q.reshape(1, -1), 0)
    assert np.array_equal(fused, unfused)


def test_predict_restarts_and_small_training_set(gpu):
    """n_restarts=2 (Hopf.py:84) and nn > rows (argsort(...)[:nn] keeps every row)."""
    import torch
    xm, ym = _nm_case(8, 3, 4)
    mdl = gpu.NNGP_p(n=3, N=4, nn=15, n_restarts=2, seed=5)
    mdl.fit(xm, ym, k=0)
    got = mdl.predict(xm[0].reshape(1, -1) + 0.01, None, None, i=0)
    th0 = np.random.default_rng(5).integers(-8, 0, (3 * 9 * 2, 2)).astype(float)
    ora = O.predict(xm, ym, xm[0] + 0.01, 8, th0, n_restarts=2)
    assert np.max(np.abs(got - ora)) <= 1e-12 * max(1e-6, np.max(np.abs(ora)))


@pytest.mark.parametrize('park', ['0', '30', '100'])
@pytest.mark.parametrize('m,d,R', [(5, 3, 1), (12, 4, 2), (16, 3, 2), (17, 5, 2), (19, 7, 1), (20, 6, 1), (20, 3, 2), (30, 2, 2),
                                   (15, 40, 1),
                                   (10, 300, 1), (18, 130, 2), (20, 80, 1), (24, 3, 1),
                                   (40, 3, 1), (48, 4, 2), (64, 3, 1), (56, 40, 1), (33, 140, 1)])
def test_predict_every_padded_size_and_fallback_vs_oracle(gpu, m, d, R, park, monkeypatch):
    """Fits run padded to 8/16/18/20/24/32/48/64 rows (identity pad, exact; m > 32 -- the adaptive
    m = max(10, k+2) past iteration 30, models.py:172-175 -- with 3-4 kernel rows per lane).  Up to 8 fits per CU each fit
    gets a wave and evaluates reflect/expand/contract points speculatively; above that (d=300:
    2 700 fits) the packed kernel runs 4 fits per wave, fused with the arg-min and mean -- or,
    when a coordinate's fits exceed a workgroup (m=18, R=2 at d=130: 4 680 fits), as fits +
    arg-min/mean kernels.  With the tail hand-off (NNGP_NM_PARK = cap > 0) the packed kernel
    parks every fit still running at `cap` evaluations and the speculative kernel resumes it
    (cap 30 parks most fits).  Up to #CU fits a fit gets four waves and up to twice that two (the
    two-level speculation: the next iteration's candidates for the likeliest outcomes; m=15 d=40:
    360 fits, two waves).  Every path is bitwise the oracle."""
    import torch
    monkeypatch.setenv('NNGP_NM_PARK', park)
    rng = np.random.default_rng(m * 10 + d + R)
    X = np.cumsum(0.05 * rng.standard_normal((3 * m, d)), axis=0)
    Y = 0.01 * np.sin(3 * X) + 1e-5 * rng.standard_normal(X.shape)
    q = X[m] + 0.01
    mdl = gpu.NNGP_p(n=d, N=4, nn=m, n_restarts=R, seed=3)
    th0 = mdl.draw_thetas(1)
    fits = torch.empty((mdl.n_fits, 4), dtype=torch.float64, device='cuda')
    bias = rng.standard_normal(d)
    out = torch.empty(d, dtype=torch.float64, device='cuda')
    preds = mdl.predict_device(_t(torch, X), _t(torch, Y), X.shape[0], _t(torch, q), _t(torch, th0),
                               fits_out=fits, out=out, bias=_t(torch, bias)).cpu().numpy()
    ora, ofits = O.predict(X, Y, q, m, th0, n_restarts=R, return_fits=True)
    assert np.array_equal(fits.cpu().numpy(), ofits)
    assert np.array_equal(preds, ora)
    assert np.array_equal(out.cpu().numpy(), ora + bias)


@pytest.mark.parametrize('d,R,world', [(3, 1, 2), (128, 1, 3), (300, 1, 8), (130, 2, 4)])
def test_predict_range_blocks_concatenate_to_predict(gpu, d, R, world):
    """nngp_predict_range over the coordinate blocks of shard_bounds (the multi-rank sweep's
    shares) concatenates to nngp_predict bit for bit -- the spec, packed and split fit paths."""
    import ctypes
    import torch
    from nngp_amd.models import JITTERS
    from nngp_amd.parareal import shard_bounds
    m = 15
    rng = np.random.default_rng(d + R)
    X = np.cumsum(0.05 * rng.standard_normal((4 * m, d)), axis=0)
    Y = 0.01 * np.sin(3 * X) + 1e-5 * rng.standard_normal(X.shape)
    q = X[m] + 0.01
    mdl = gpu.NNGP_p(n=d, N=4, nn=m, n_restarts=R, seed=3)
    th0 = _t(torch, mdl.draw_thetas(1))
    Xt, Yt, qt = _t(torch, X), _t(torch, Y), _t(torch, q)
    full = mdl.predict_device(Xt, Yt, X.shape[0], qt, th0).cpu().numpy()
    jit = np.ascontiguousarray(JITTERS)
    parts = []
    for r in range(world):
        c0, c1, _ = shard_bounds(0, d, world, r)
        if c1 <= c0:
            continue
        out = torch.empty(c1 - c0, dtype=torch.float64, device='cuda')
        gpu._lib.check(gpu.lib().nngp_predict_range(
            Xt.data_ptr(), Yt.data_ptr(), X.shape[0], d, qt.data_ptr(), m, len(jit),
            jit.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), R, th0.data_ptr(), c0, c1, 0.1, 0.1, 400,
            out.data_ptr(), None))
        parts.append(out.cpu().numpy())
    assert np.array_equal(np.concatenate(parts), full)


@pytest.mark.parametrize('nx,n_slices,norm', [(20, 512, False), (20, 64, True), (22, 8, False)])
def test_fhn_pde_full_size_vs_oracle(gpu, nx, n_slices, norm):
    """BASELINE configs[4]'s FHN-PDE at its full size (d = 2*20^2 = 800, 512 slices; the 8-GPU
    share of 64 slices; and d = 968 near the 512-thread form's limit), RK8: sampled slices are
    bitwise the oracle's."""
    import torch
    ode = gpu.FHN_PDE(d_x=nx, normalization='-11' if norm else None)
    s = gpu.SolverRK(ode.get_vector_field(), Ng=1, Nf=6, F='RK8', G='RK1')
    rng = np.random.default_rng(nx + n_slices)
    U0 = np.clip(ode.get_init_cond()[None, :] + 0.01 * rng.standard_normal((n_slices, ode.d)), -1, 1)
    T = np.arange(n_slices + 1) * 6e-3      # 1e-3 per RK8 step: inside the explicit stability region
    out = s.run_F_batch(_t(torch, T[:-1]), _t(torch, T[1:]), _t(torch, U0)).cpu().numpy()
    so = O.System('fhn_pde', nx=nx, mn=-1, mx=1) if norm else O.System('fhn_pde', nx=nx, normalized=False)
    assert np.all(np.isfinite(out))
    for i in sorted({0, 1, n_slices // 2, n_slices - 1}):
        assert np.array_equal(out[i], so.rk(8, T[i], T[i + 1], 6, U0[i], O.STEP_FIXED)), i


@pytest.mark.parametrize('d,w4,w2,n400', [(150, None, None, 250), (150, '0', '0', 250), (150, '0', '100000', 250),
                                         (150, '100000', '100000', 250), (20, None, None, 40), (50, None, None, 90)])
def test_predict_parked_all_inf_fits_vs_oracle(gpu, d, w4, w2, n400, monkeypatch):
    """Exactly duplicated training rows make K + jitter*I singular in floating point for the jitters
    <= 1e-16 (1 + j == 1): those fits' simplices are all +inf and run to maxfev = 400, like the
    parked tail of a real FHN-PDE d = 800 correction.
    - d = 150, m = 20 (1 350 fits, the packed kernel): fits still running at 70 evaluations are
      parked, the finite ones at the front of the park list and the all-+inf ones at its back.
      The resume gives a finite fit 4 waves of the two-level kernel (default: up to #CU of them;
      NNGP_RESUME_W4/W2 = 100000 forces it), 2 (W4 = 0, W2 = 100000) or 1 (both 0: the one-level
      kernel), and an all-+inf fit one wave.
    - d = 20 / 50 (180 / 450 fits: the two-level kernel from the start, 4 / 2 waves per fit): an
      all-+inf simplex takes W whole iterations per round -- each wave answers the requests the
      state machine makes if the earlier ones are +inf too.
    Every case is bitwise the oracle."""
    import torch
    for k, v in (('NNGP_RESUME_W4', w4), ('NNGP_RESUME_W2', w2)):
        if v is not None:
            monkeypatch.setenv(k, v)
    m = 20
    rng = np.random.default_rng(150)
    base = np.cumsum(0.005 * rng.standard_normal((40, d)), axis=0)
    X = np.repeat(base, 4, axis=0)          # every state 4 times: duplicated kernel rows
    Y = np.sin(3 * X) + 1e-5 * rng.standard_normal(X.shape)
    q = X[30] + 0.01
    mdl = gpu.NNGP_p(n=d, N=4, nn=m, n_restarts=1, seed=9)
    th0 = mdl.draw_thetas(1)
    fits = torch.empty((mdl.n_fits, 4), dtype=torch.float64, device='cuda')
    preds = mdl.predict_device(_t(torch, X), _t(torch, Y), X.shape[0], _t(torch, q), _t(torch, th0),
                               fits_out=fits).cpu().numpy()
    ora, ofits = O.predict(X, Y, q, m, th0, return_fits=True)
    f = fits.cpu().numpy()
    assert (f[:, 3] >= 400).sum() >= n400   # fits that ran to maxfev (d = 150: 304 of 1 350; 716 parked)
    assert np.array_equal(f, ofits)
    assert np.array_equal(preds, ora)


def test_predict_fhn_pde_d800_vs_oracle(gpu):
    """BASELINE configs[4]'s correction shape: FHN-PDE d = 800, m = 20, R = 1 (FHN_PDE.py:175-176):
    7 200 fits per prediction -- the packed fits kernel with the tail hand-off (fits still running
    at 70 evaluations are parked and finished by the speculative kernel), then the arg-min + mean
    kernel -- bitwise the oracle's fits and prediction."""
    import torch
    d, rows, m = 800, 1500, 20
    rng = np.random.default_rng(800)
    X = np.clip(np.cumsum(0.01 * rng.standard_normal((rows, d)), axis=0), -1, 1)
    Y = 0.02 * np.sin(2 * X) + 1e-5 * rng.standard_normal(X.shape)
    q = X[rows // 3] + 1e-3
    mdl = gpu.NNGP_p(n=d, N=4, nn=m, n_restarts=1, seed=45)
    th0 = mdl.draw_thetas(1)
    assert mdl.n_fits == 7200
    fits = torch.empty((mdl.n_fits, 4), dtype=torch.float64, device='cuda')
    bias = rng.standard_normal(d)
    out = torch.empty(d, dtype=torch.float64, device='cuda')
    preds = mdl.predict_device(_t(torch, X), _t(torch, Y), rows, _t(torch, q), _t(torch, th0), fits_out=fits,
                               out=out, bias=_t(torch, bias)).cpu().numpy()
    ora, ofits = O.predict(X, Y, q, m, th0, return_fits=True)
    f = fits.cpu().numpy()
    assert np.array_equal(f, ofits)
    assert np.array_equal(preds, ora)
    assert np.array_equal(out.cpu().numpy(), ora + bias)
    print('FHN-PDE d=800 nfev mean %.1f max %d' % (f[:, 3].mean(), f[:, 3].max()))
