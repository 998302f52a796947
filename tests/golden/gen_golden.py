"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

Run in the development container only (the reference tree and this script never travel to the
GPU box; only the .npz outputs are committed and used by the tests):

    PYTHONPATH=tests/golden/jaxshim:/root/reference python tests/golden/gen_golden.py <part> ...

jax is not installed here, so `tests/golden/jaxshim` (our own numpy stand-in) lets the reference
modules import and run in fp64.  Every number written below is
computed by reference code (systems.py, RK.py, solver.py, models.py, parareal.py, new_lib.py);
this script only chooses inputs and records outputs.  One documented speed substitution: the
shim's python-loop `vmap` is replaced by a broadcast squared-exponential kernel with the same
numpy reduction (pairwise sum over the contiguous last axis), so values are unchanged.

Parts: rhs rk lml nm knn preds para_lorenz para_fhn para_burgers legacy gp rng
"""
import os
import sys
import time
import itertools

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

import systems as rsys          # noqa: E402  (reference)
import RK as rrk                # noqa: E402
import solver as rsolver        # noqa: E402
import models as rmodels        # noqa: E402
import parareal as rpara        # noqa: E402


def _broadcast_kernel(x, y, kernel_params):
    sigma_x, sigma_y = kernel_params
    x = np.asarray(x, dtype=float)
    y = np.asarray(y, dtype=float)
    sq = ((x[:, None, :] - y[None, :, :]) ** 2).sum(-1)
    return 10 ** (sigma_y) * np.exp(-0.5 * (1 / (10 ** sigma_x)) * sq)


rmodels.NNGP_p.kernel_jit = staticmethod(_broadcast_kernel)


def save(name, **arrs):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrs)
    print('wrote', path, {k: np.shape(v) for k, v in arrs.items()}, flush=True)


# ----------------------------------------------------------------------------------------------
# systems used throughout (reference constructors, modern API)
# ----------------------------------------------------------------------------------------------
def make_systems():
    out = {}
    out['lorenz'] = rsys.Lorenz(normalization='-11')
    out['hopf'] = rsys.Hopf(normalization='-11')
    out['tomlab'] = rsys.ThomasLabyrinth(normalization='-11')
    out['fhn_ode'] = rsys.FHN_ODE(normalization='-11')
    out['rossler'] = rsys.Rossler(normalization='-11')
    out['brus'] = rsys.Brusselator(normalization='-11')
    out['dblpend'] = rsys.DblPend(normalization='-11')
    out['lorenz_id'] = rsys.Lorenz()
    out['burgers128'] = rsys.Burgers(d_x=128, normalization='-11')
    out['burgers16'] = rsys.Burgers(d_x=16, normalization='-11')
    out['fhnpde10'] = rsys.FHN_PDE(d_x=10)
    out['fhnpde10_n'] = rsys.FHN_PDE(d_x=10, normalization='-11')
    out['fhnpde4'] = rsys.FHN_PDE(d_x=4)
    return out


def part_rhs():
    rng = np.random.default_rng(1234)
    arrs = {}
    for name, ode in make_systems().items():
        f = ode.get_vector_field()
        d = ode.get_dim()
        U = rng.uniform(-0.9, 0.9, size=(4, d))
        U[0] = ode.get_init_cond()
        F = np.stack([np.asarray(f(0.0, u), dtype=float) for u in U])
        arrs[name + '__u'] = U
        arrs[name + '__f'] = F
        arrs[name + '__u0'] = ode.get_init_cond()
    save('rhs.npz', **arrs)


def part_rk():
    """Single-slice propagations, RK.run_get_last (fixed dt, RK.py:101-109) and RK.run (linspace
    grid, RK.py:91-99, the legacy new_lib.RK convention)."""
    rng = np.random.default_rng(99)
    arrs = {}
    cases = [('lorenz', 0.0, 0.5625, 40), ('hopf', -20.0, -15.9375, 30), ('tomlab', 0.0, 0.3125, 30),
             ('fhn_ode', 0.0, 1.0, 25), ('rossler', 0.0, 1.0, 20), ('brus', 0.0, 1.0, 20),
             ('dblpend', 0.0, 0.5, 20), ('burgers16', 0.0, 0.05, 20), ('burgers128', 0.0, 0.0390625, 20),
             ('fhnpde4', 0.0, 0.2, 10), ('fhnpde10', 0.0, 0.2, 10), ('fhnpde10_n', 0.0, 0.2, 10)]
    systems_ = make_systems()
    for name, t0, t1, steps in cases:
        ode = systems_[name]
        f = ode.get_vector_field()
        d = ode.get_dim()
        u0 = ode.get_init_cond() + rng.uniform(-0.02, 0.02, size=d)
        u0 = np.clip(u0, -1, 1) if 'burgers' not in name else u0
        for tab in ['RK1', 'RK2', 'RK4', 'RK8']:
            r = rrk.RK(f, tab)
            st = time.time()
            last = np.asarray(r.run_get_last(t0, t1, steps, u0), dtype=float)
            full = np.asarray(r.run(t0, t1, steps, u0), dtype=float)[-1]
            key = f'{name}__{tab}'
            arrs[key + '__u0'] = u0
            arrs[key + '__span'] = np.array([t0, t1, steps], dtype=float)
            arrs[key + '__fixed'] = last
            arrs[key + '__linspace'] = full
            print(key, f'{time.time()-st:.1f}s', flush=True)
    # paged propagation (solver.py:86-99 quirk): thresh < steps
    ode = systems_['lorenz']
    s = rsolver.SolverRK(ode.get_vector_field(), Ng=6, Nf=45, F='RK4', G='RK4', thresh=10)
    u0 = ode.get_init_cond()
    arrs['paged__lorenz__u0'] = u0
    arrs['paged__lorenz__args'] = np.array([0.0, 0.5625, 45, 10], dtype=float)
    arrs['paged__lorenz__out'] = np.asarray(s.run_F(0.0, 0.5625, u0), dtype=float)
    s = rsolver.SolverRK(ode.get_vector_field(), Ng=6, Nf=45, F='RK4', G='RK4', thresh=7.3)
    arrs['paged73__lorenz__args'] = np.array([0.0, 0.5625, 45, 7.3], dtype=float)
    arrs['paged73__lorenz__out'] = np.asarray(s.run_F(0.0, 0.5625, u0), dtype=float)
    save('rk.npz', **arrs)


def _lorenz_training_set(m=10, seed=0):
    rng = np.random.default_rng(seed)
    x = rng.uniform(-0.8, 0.8, size=(60, 3))
    y = 0.05 * np.sin(3 * x) + 1e-3 * rng.normal(size=x.shape)
    new_x = rng.uniform(-0.5, 0.5, size=(1, 3))
    return x, y, new_x


def part_lml():
    """-LML (models.py:240-252) over a grid of (theta, jitter), including Cholesky failures (inf)."""
    arrs = {}
    x, y, new_x = _lorenz_training_set()
    xm, ym = x[:12], y[:12]
    thetas = np.array(list(itertools.product(np.arange(-8, 3, 1.0), np.arange(-8, 3, 1.0))))
    jitters = np.arange(-20, -11, dtype=float)
    vals = np.empty((len(jitters), len(thetas), 3))
    for a, jit in enumerate(jitters):
        for b, th in enumerate(thetas):
            for j in range(3):
                vals[a, b, j] = rmodels.NNGP_p.log_lik(xm, ym[:, j], th, jit, rmodels.NNGP_p.kernel_jit)
    arrs['xm'], arrs['ym'], arrs['thetas'], arrs['jitters'], arrs['nlml'] = xm, ym, thetas, jitters, vals
    # duplicated rows (singular kernel w/o jitter)
    xd = np.vstack([xm[:6], xm[:6]])
    yd = np.vstack([ym[:6], ym[:6]])
    vd = np.empty((len(jitters), len(thetas)))
    for a, jit in enumerate(jitters):
        for b, th in enumerate(thetas):
            vd[a, b] = rmodels.NNGP_p.log_lik(xd, yd[:, 0], th, jit, rmodels.NNGP_p.kernel_jit)
    arrs['xd'], arrs['yd'], arrs['nlml_dup'] = xd, yd, vd
    # posterior means (models.py:162-168)
    pm = np.empty((len(thetas), 3))
    for b, th in enumerate(thetas):
        for j in range(3):
            pm[b, j] = np.squeeze(rmodels.NNGP_p._predict(xm, ym[:, j], th, rmodels.NNGP_p.kernel_jit, -15.0, new_x))
    arrs['new_x'], arrs['post_mean_jit15'] = new_x, pm
    save('lml.npz', **arrs)


def _nm_fit(xm, y, theta0, jitter, fatol, xatol):
    from scipy.optimize import minimize
    f = lambda th: rmodels.NNGP_p.log_lik(xm, y, th, jitter, rmodels.NNGP_p.kernel_jit)
    res = minimize(f, theta0, method='Nelder-Mead', options={'fatol': fatol, 'xatol': xatol})
    return np.array(res.x, dtype=float), float(res.fun), int(res.nfev), int(res.nit)


def part_nm():
    """scipy Nelder-Mead on -LML (models.py:254-260): theta, fval, nfev, nit per fit."""
    arrs = {}
    rng = np.random.default_rng(7)
    x, y, new_x = _lorenz_training_set(seed=3)
    for tag, m, fatol, xatol in [('m10', 10, 0.1, 0.1), ('m18tol3', 18, 1e-3, 1e-3), ('m30', 30, 0.1, 0.1)]:
        xm, ym = x[:m], y[:m]
        ins = list(itertools.product(range(3), np.arange(-20, -11, dtype=float), range(1)))
        th0 = rng.integers(-8, 0, (len(ins), 2))
        out = np.empty((len(ins), 5))
        for q, (j, jit, _) in enumerate(ins):
            th, fv, nfev, nit = _nm_fit(xm, ym[:, j], th0[q], jit, fatol, xatol)
            out[q] = [th[0], th[1], fv, nfev, nit]
        arrs[tag + '__xm'], arrs[tag + '__ym'] = xm, ym
        arrs[tag + '__ins'] = np.array([[j, jit] for j, jit, _ in ins])
        arrs[tag + '__th0'] = th0.astype(float)
        arrs[tag + '__tol'] = np.array([fatol, xatol])
        arrs[tag + '__out'] = out
        print('nm', tag, 'done', flush=True)
    save('nm.npz', **arrs)


def part_knn():
    import scipy.spatial
    rng = np.random.default_rng(11)
    X = rng.normal(size=(500, 5))
    X[100] = X[7]          # exact duplicate -> tie
    q = rng.normal(size=(1, 5))
    dist = scipy.spatial.distance.cdist(q, X, metric='sqeuclidean')[0]
    idx = np.argsort(dist)
    save('knn.npz', X=X, q=q, dist=dist, idx=idx)


class RecordingPool:
    """A MyPool (parareal.py:16-24) that records every NNGP fit fan-out (models.py:197-202)."""
    def __init__(self, limit=4):
        self.calls = []
        self.limit = limit

    def map(self, fn, *its, **kw):
        its = [list(i) if not isinstance(i, itertools.repeat) else i for i in its]
        res = list(map(fn, *its))
        if getattr(fn, '__name__', '') == '_get_opt_par' and len(self.calls) < self.limit:
            static, ins, rnd = its
            st = next(static)
            self.calls.append(dict(xm=st[0], ym=st[1], tol=np.array(st[2:4]), ins=np.array([[i[0], i[1], i[2]] for i in ins]),
                                   rnd=np.array(rnd, dtype=float), res=np.array([r[:-1] for r in res], dtype=float)))
        return iter(res)

    def shutdown(self, *a, **k):
        pass


def _run_para(ode, cfg, model, N=None, **kw):
    f = ode.get_vector_field()
    s = rsolver.SolverRK(f, Ng=cfg['Ng'], Nf=cfg['Nf'], F=cfg['F'], G=cfg['G'])
    p = rpara.Parareal(ode, s, tspan=cfg['tspan'], N=N or cfg['N'], epsilon=cfg.get('eps', 5e-7), verbose=None)
    pool = kw.pop('pool', None)
    st = time.time()
    res = p.run(model=model, pool=pool, **kw)
    print(model, kw.get('seed'), 'K=', res['k'], f'{time.time()-st:.1f}s', flush=True)
    return res


def _dump_run(prefix, res, arrs):
    arrs[prefix + '__k'] = np.array(res['k'])
    arrs[prefix + '__conv_int'] = np.array(res['conv_int'])
    arrs[prefix + '__u'] = res['u']
    arrs[prefix + '__err'] = res['err']
    arrs[prefix + '__converged'] = np.array(res['converged'])


def part_para_lorenz():
    """BASELINE configs[0]: Lorenz N=32, tspan [0,18], G=RK4 6/slice, F=RK4 450/slice, eps 5e-7."""
    cfg = dict(tspan=[0, 18], N=32, Ng=6, Nf=450, F='RK4', G='RK4', eps=5e-7)
    arrs = {}
    ode = rsys.Lorenz(normalization='-11')
    arrs['cfg'] = np.array([0, 18, 32, 6, 450, 5e-7])
    res = _run_para(ode, cfg, 'parareal')
    _dump_run('para', res, arrs)
    for seed in [45, 46, 47, 48, 49]:
        pool = RecordingPool(limit=2 if seed == 45 else 0)
        res = _run_para(ode, cfg, 'nngp', pool=pool, nn=10, seed=seed)
        _dump_run(f'nngp_s{seed}', res, arrs)
        for c, call in enumerate(pool.calls):
            for k2, v in call.items():
                arrs[f'call{c}__{k2}'] = v
    # serial fine reference at the slice boundaries (for final-state error)
    f = ode.get_vector_field()
    r = rrk.RK(f, 'RK4')
    t = np.linspace(0, 18, 33)
    u = ode.get_init_cond()
    fine = [u]
    for i in range(32):
        u = np.asarray(r.run_get_last(t[i], t[i + 1], 450, u), dtype=float)
        fine.append(u)
    arrs['fine'] = np.array(fine)
    save('para_lorenz.npz', **arrs)


def part_para_fhn():
    """FHN-ODE (configs.py:7-16): N=40, G=RK2 4/slice, F=RK4 4000/slice; nnGP m=15 and Parareal."""
    cfg = dict(tspan=[0, 40], N=40, Ng=4, Nf=4000, F='RK4', G='RK2', eps=5e-7)
    arrs = {}
    ode = rsys.FHN_ODE(normalization='-11')
    arrs['cfg'] = np.array([0, 40, 40, 4, 4000, 5e-7])
    res = _run_para(ode, cfg, 'parareal')
    _dump_run('para', res, arrs)
    res = _run_para(ode, cfg, 'nngp', nn=15, seed=45)
    _dump_run('nngp_s45', res, arrs)
    f = ode.get_vector_field()
    r = rrk.RK(f, 'RK4')
    t = np.linspace(0, 40, 41)
    u = ode.get_init_cond()
    fine = [u]
    for i in range(40):
        u = np.asarray(r.run_get_last(t[i], t[i + 1], 4000, u), dtype=float)
        fine.append(u)
    arrs['fine'] = np.array(fine)
    save('para_fhn.npz', **arrs)


def part_preds():
    """One full NNGP_p.predict (models.py:171-226) at d=128 on Parareal-like training data: states
    along a Burgers trajectory (x) and their fine-minus-coarse corrections (y), m=15."""
    import concurrent.futures
    ode = rsys.Burgers(d_x=128, normalization='-11')
    f = ode.get_vector_field()
    rF, rG = rrk.RK(f, 'RK8'), rrk.RK(f, 'RK1')
    dt = 5 / 128
    u = ode.get_init_cond()
    X, Y = [], []
    for i in range(40):
        uf = np.asarray(rF.run_get_last(0.0, dt, 40, u), dtype=float)
        ug = np.asarray(rG.run_get_last(0.0, dt, 4, u), dtype=float)
        X.append(u)
        Y.append(uf - ug)
        u = ug + 0.999 * (uf - ug)     # a nearby, not identical, next state
    X, Y = np.array(X), np.array(Y)
    new_x = (0.5 * (X[20] + X[21])).reshape(1, -1)
    pool = RecordingPool(limit=1)
    mdl = rmodels.NNGP_p(n=128, N=8, worker_pool=pool, nn=15, seed=45)
    mdl.fit(X, Y, k=0)
    st = time.time()
    preds = mdl.predict(new_x, None, None, i=0)
    print('preds d=128', f'{time.time()-st:.1f}s', flush=True)
    c = pool.calls[0]
    save('preds_d128.npz', X=X, Y=Y, new_x=new_x, m=np.array(15), seed=np.array(45), preds=preds,
         fit_res=c['res'], rnd=c['rnd'], xm=c['xm'], ym=c['ym'])


def part_legacy():
    """The legacy monolith (new_lib.Parareal, the API of every published scalability run): total
    step counts, per-slice np.linspace grids, one global initial coarse grid, and RK_last's paging
    quirk with float page lengths (RK_thresh = Nf/N/2.5 -> pages of 180, 180, 90 step-units, each
    re-using the full 450-step count)."""
    import new_lib as rnl
    rnl.NNGP_p.kernel_jit = staticmethod(_broadcast_kernel)   # same speed substitution as above
    arrs = {}
    s = rnl.Parareal(ode_name='lorenz_n', epsilon=5e-7, verbose=None)
    s.RK_thresh = s.Nf / s.N / 2.5
    st = time.time()
    res = s.run(model='parareal')
    print('legacy parareal paged K=', res['k'], f'{time.time()-st:.1f}s', flush=True)
    _dump_run('lorenz_para_paged', res, arrs)
    s = rnl.Parareal(ode_name='lorenz_n', epsilon=5e-7, verbose=None)
    st = time.time()
    res = s.run(model='nngp', nn=10, seed=45, early_stop=3)
    print('legacy nngp 3 iterations', f'{time.time()-st:.1f}s', flush=True)
    _dump_run('lorenz_nngp3', res, arrs)
    save('legacy.npz', **arrs)


class GPRecordingPool(RecordingPool):
    """Records the first `limit` GPjax_p._train fan-outs (models.py:404-407): static inputs
    (x, y, old thetas, fatol, xatol), the (coordinate, jitter) list and every fit's result."""
    def map(self, fn, *its, **kw):
        its = [list(i) if not isinstance(i, itertools.repeat) else i for i in its]
        res = list(map(fn, *its))
        if getattr(fn, '__name__', '') == '_get_opt_par' and len(self.calls) < self.limit:
            static, ins = its
            st = next(static)
            self.calls.append(dict(x=np.asarray(st[0]), y=np.asarray(st[1]), old=np.asarray(st[2], dtype=float),
                                   tol=np.array(st[3:5], dtype=float), ins=np.array(ins, dtype=float),
                                   res=np.array([r[:-1] for r in res], dtype=float)))
        return iter(res)


def part_gp():
    """Full-data GParareal (model='gpjax', models.py:273-473) on BASELINE configs[0] (Lorenz N=32),
    default tolerances (fatol = xatol = 1e-4); records the first two training fan-outs and a few
    log-likelihood values (GPjax_p.log_lik, models.py:321-327) on the recorded data."""
    cfg = dict(tspan=[0, 18], N=32, Ng=6, Nf=450, F='RK4', G='RK4', eps=5e-7)
    arrs = {}
    ode = rsys.Lorenz(normalization='-11')
    pool = GPRecordingPool(limit=2)
    res = _run_para(ode, cfg, 'gpjax', pool=pool)
    _dump_run('gp', res, arrs)
    for c, call in enumerate(pool.calls):
        for k2, v in call.items():
            arrs[f'call{c}__{k2}'] = v
    rng = np.random.default_rng(3)
    c1 = pool.calls[-1]
    th = np.concatenate([10 ** rng.uniform(-2, 1, (6, 2)), [[1.0, 1.0], [1e-3, 5.0]]])
    jit = np.array([-20., -16., -12., -13., -20., -11., -15., -20.])
    lml = np.array([rmodels.GPjax_p.log_lik(c1['x'], c1['y'][:, j % 3], th[j], jit[j]) for j in range(len(th))])
    arrs['lml_theta'], arrs['lml_jitter'], arrs['lml_val'] = th, jit, lml
    save('gp_lorenz.npz', **arrs)


def part_gp_fhn():
    """Full-data GParareal on FHN-ODE (configs.py:7-16: N=40, G=RK2 4/slice, F=RK4 4000/slice),
    a non-chaotic case for exact-K parity."""
    cfg = dict(tspan=[0, 40], N=40, Ng=4, Nf=4000, F='RK4', G='RK2', eps=5e-7)
    arrs = {}
    ode = rsys.FHN_ODE(normalization='-11')
    res = _run_para(ode, cfg, 'gpjax', pool=GPRecordingPool(limit=0))
    _dump_run('gp', res, arrs)
    save('gp_fhn.npz', **arrs)


def part_rng():
    rng = np.random.default_rng(45)
    a = np.array([rng.integers(-8, 0, 2) for _ in range(300)])
    save('rng.npz', draws=a)


if __name__ == '__main__':
    parts = sys.argv[1:] or ['rhs', 'rk', 'lml', 'nm', 'knn', 'rng']
    for p in parts:
        st = time.time()
        globals()['part_' + p]()
        print('part', p, f'{time.time()-st:.1f}s', flush=True)
