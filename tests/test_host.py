"""CPU: host-side logic of the product package (no GPU calls)."""
import os

import numpy as np
import pytest

from conftest import ROOT, golden


def test_vectorised_draws_equal_the_reference_draw_loop():
    """models.py:192 draws rng.integers(-8, 0, 2) once per fit; one vectorised call over a whole
    iteration yields the same stream (power-of-two range: Lemire never rejects)."""
    g = golden('rng.npz')['draws']
    rng = np.random.default_rng(45)
    assert np.array_equal(rng.integers(-8, 0, (len(g), 2)), g)


def test_nngp_model_draw_order_matches_reference_predictions():
    import nngp_amd
    m = nngp_amd.NNGP_p(n=3, N=8, nn=10, seed=45)
    a = m.draw_thetas(2)              # two consecutive predictions of 27 fits each
    ref = np.random.default_rng(45)
    exp = np.array([ref.integers(-8, 0, 2) for _ in range(54)], dtype=float)
    assert np.array_equal(a, exp)
    assert m.n_fits == 27 and m.maxfev == 400


def test_adaptive_neighbours():
    import nngp_amd
    m = nngp_amd.NNGP_p(n=3, N=8, nn='adaptive')
    m.k = 3
    assert m.n_neighbours() == 10
    m.k = 20
    assert m.n_neighbours() == 22


@pytest.mark.parametrize('key,factory', [
    ('lorenz', lambda g: g.Lorenz(normalization='-11')),
    ('hopf', lambda g: g.Hopf(normalization='-11')),
    ('tomlab', lambda g: g.ThomasLabyrinth(normalization='-11')),
    ('burgers128', lambda g: g.Burgers(d_x=128, normalization='-11')),
    ('fhnpde10', lambda g: g.FHN_PDE(d_x=10)),
    ('fhnpde10_n', lambda g: g.FHN_PDE(d_x=10, normalization='-11')),
])
def test_initial_conditions_match_reference(key, factory):
    import nngp_amd
    R = golden('rhs.npz')
    assert np.array_equal(factory(nngp_amd).get_init_cond(), R[key + '__u0'])


def test_normalisation_table():
    import nngp_amd
    o = nngp_amd.Lorenz(normalization='-11')
    t = o.normalizer.device_table(3)
    mn, mx = np.array([-17.1, -23, 6]), np.array([18.1, 25, 45])
    assert np.array_equal(t, np.concatenate([mn, mx - mn, 2 / (mx - mn)]))
    assert nngp_amd.Lorenz().normalizer.device_table(3) is None


def test_configs_restate_reference():
    import nngp_amd
    c = nngp_amd.Config(nngp_amd.Lorenz(normalization='-11')).get()
    assert (c['N'], c['Ng'], c['Nf'], c['G'], c['F']) == (50, 6, 450, 'RK4', 'RK4')
    c = nngp_amd.Config(nngp_amd.Hopf(normalization='-11'), N=128).get()
    assert (c['Ng'], c['Nf'], c['G'], c['F']) == (16, 1360, 'RK1', 'RK8')
    c = nngp_amd.Config(nngp_amd.ThomasLabyrinth(normalization='-11'), N=256).get()
    assert (c['Ng'], c['Nf'], c['tspan']) == (10, 3910, [0, 100])
    c = nngp_amd.Config(nngp_amd.FHN_PDE(d_x=10), d_x=10).get()
    assert (c['N'], c['Ng'], c['Nf'], c['G'], c['F'], c['tspan']) == (512, 3, 21, 'RK2', 'RK8', [0, 150])


def test_paging_schedule_restates_solver_quirk():
    from nngp_amd.solver import _paging_schedule
    assert _paging_schedule(45, 10) == ([10, 10, 10, 10, 4], 44)
    it, st = _paging_schedule(45, 7.3)
    assert st == 44 and len(it) == 7 and abs(it[-1] - 44 % 7.3) < 1e-15


def test_solver_rejects_unknown_tableau():
    import nngp_amd
    f = nngp_amd.Lorenz().get_vector_field()
    with pytest.raises(NotImplementedError):
        nngp_amd.SolverRK(f, 6, 45, 'RK3', 'RK4')
    with pytest.raises(TypeError):
        nngp_amd.SolverRK(lambda t, u: u, 6, 45, 'RK4', 'RK4')


def test_contracted_propagator_is_opt_in(monkeypatch):
    """SolverRK(fma=True) ORs NNGP_STEP_CONTRACT (include/nngp.h) onto either step convention; the
    default is the exact build unless NNGP_RK_CONTRACT=1."""
    import nngp_amd
    f = nngp_amd.Lorenz().get_vector_field()
    monkeypatch.delenv('NNGP_RK_CONTRACT', raising=False)
    assert nngp_amd.SolverRK(f, 6, 45, 'RK4', 'RK4').step_mode == 0
    assert nngp_amd.SolverRK(f, 6, 45, 'RK4', 'RK4', fma=True).step_mode == 16
    assert nngp_amd.SolverRK(f, 6, 45, 'RK4', 'RK4', step_mode='linspace', fma=True).step_mode == 17
    monkeypatch.setenv('NNGP_RK_CONTRACT', '1')
    assert nngp_amd.SolverRK(f, 6, 45, 'RK4', 'RK4').fma
    assert not nngp_amd.SolverRK(f, 6, 45, 'RK4', 'RK4', fma=False).fma


def test_store_int_checkpoint_round_trip_without_gpu(tmp_path):
    """Checkpoints are npz + JSON (numpy safe loader, no pickle): arrays, scalars and the
    model's RNG state survive a round trip, and the restored RNG continues the same stream."""
    import nngp_amd
    ode = nngp_amd.Lorenz(normalization='-11')
    s = nngp_amd.SolverRK(ode.get_vector_field(), Ng=6, Nf=45, F='RK4', G='RK4')
    p = nngp_amd.Parareal(ode, s, [0, 18], 4, verbose=None)
    mdl = nngp_amd.NNGP_p(n=3, N=4, nn=10, seed=47)
    mdl.draw_thetas(2)
    objs = {'I': 2, 'k': 1, 'conv_int': np.array([1, 2]), 'u': np.arange(30.0).reshape(5, 3, 2),
            'G_time': 0.5, 'F_time': np.float64(1.5)}
    p.store(name='ck', path=str(tmp_path), mdl=mdl, objs=objs)
    st = p.read_int_dump(str(tmp_path / 'ck'))
    assert st['I'] == 2 and st['k'] == 1 and st['F_time'] == 1.5 and st['ode_name'] == 'Lorenz'
    assert np.array_equal(st['u'], objs['u']) and list(st['conv_int']) == [1, 2]
    m2 = nngp_amd.NNGP_p(n=3, N=4, **st['model']['settings'])
    m2.load_state(st['model'])
    assert np.array_equal(m2.draw_thetas(3), mdl.draw_thetas(3))
    with np.load(str(tmp_path / 'ck.npz'), allow_pickle=False) as z:   # loadable without pickle
        assert 'meta' in z.files


def test_legacy_systems_registry_restates_new_lib():
    import nngp_amd
    f, tspan, u0, eps, N, Ng, Nf, G, F, tr, tr_inv = nngp_amd.legacy.Systems('lorenz_n').fetch()
    assert (tspan, eps, N, Ng, Nf, G, F) == ([0, 18], 1e-8, 50, 300, 22500, 'RK4', 'RK4')
    assert np.allclose(tr_inv(u0), [-15, -15, 20])
    f, tspan, u0, eps, N, Ng, Nf, G, F, _, _ = nngp_amd.legacy.Systems('non_aut128_n').fetch()
    assert (tspan, N, Ng, Nf, G, F) == ([-20, 500], 128, 2048, 174080, 'RK1', 'RK8')
    with pytest.raises(Exception):
        nngp_amd.legacy.Systems('nosuch')
    # RK_last's paging schedule (new_lib.py:59-66) incl. a float remainder page
    from nngp_amd.legacy import _legacy_pages
    assert _legacy_pages(451, 1e7) is None
    iters, pts = _legacy_pages(451, 450 / 2.5)
    assert pts == 450 and iters == [180.0, 180.0, 90.0]
    with pytest.raises(Exception):
        nngp_amd.legacy.LegacySolverRK(f, 7, 100, 1000, 'RK4', 'RK1')   # Ng % N != 0


def test_gp_fit_selection_semantics():
    """GPjax_p's per-coordinate choice (models.py:388-395): fits below 0.9*min (all if none),
    then Python's min by fval -- first minimum, NaN never chosen unless first, +inf loses."""
    from nngp_amd.models import _select_fit
    th = np.arange(18, dtype=float).reshape(9, 2)
    jit = np.arange(-20, -11, dtype=float)
    f = np.array([5.0, -3.0, -10.0, -10.0, np.inf, -1.0, 0.0, 2.0, -9.5])
    assert _select_fit(th, f, jit) == ((4.0, 5.0), -10.0, -18.0)     # first of the tied minima
    f = np.array([3.0, 2.0, 1.0, 1.0, 4.0, 5.0, 6.0, 7.0, 8.0])        # positive: mask empty -> all
    assert _select_fit(th, f, jit)[1:] == (1.0, -18.0)
    f = np.array([np.inf] * 9)
    assert np.isinf(_select_fit(th, f, jit)[1])
    f = np.array([np.nan, -5.0, -6.0] + [0.0] * 6)                     # NaN first: kept (min semantics)
    assert _select_fit(th, f, jit)[2] == -20.0


def test_report_tables_layout():
    """print_times / print_speedup (parareal.py:636-758) on recorded run timings (host only)."""
    import nngp_amd as g
    p = g.Parareal.__new__(g.Parareal)
    p.N = 32
    p.runs = {'NNGP': {'k': 19, 'timings': {'G_time': 0.01, 'F_time': 0.05, 'mdl_train_t': 0.0, 'mdl_pred_t': 0.2,
                                            'mdl_tot_t': 0.2, 'runtime': 0.3}}}
    p.fine, p.fine_t = object(), 2.0
    t = p.print_times(expected_fine=3.0).split('\n')
    assert t[0].startswith('|Model|K |') and t[0].rstrip().endswith('E[Speedup]|')
    assert '6.67' in t[3] and '1.51' in t[3]          # 2.0/0.3 and 3/(3/32*19 + 0.2)
    s = p.print_speedup(fine_t=1.5).split('\n')
    assert s[0] == '$N=32$' and s[-1] == '|NN-GParareal | 19 | 5.26e-04 | 2.63e-03 | 2.00e-01 | 3.00e-01 | 5.00|'
    x = p.print_speedup(F_t=0.1, md=False, mdl_title='Lorenz').split('\n')
    assert x[0] == r'\caption*{Lorenz, $N=32$}' and x[3] == r'\hline\\'
    assert x[-3].endswith('& ' + f'{3.2 / (0.1 * 19 + 0.2):.2f}' + r'\\')


def test_nngp_neighbour_bound_is_explicit():
    """The GPU fits support m <= 64 neighbours: an explicit nn beyond that is refused at
    construction, and nn='adaptive' (m = max(10, k+2), models.py:172-175) raises a clear error
    once k+2 passes it, instead of failing inside a kernel launch."""
    import nngp_amd
    with pytest.raises(ValueError):
        nngp_amd.NNGP_p(n=3, N=100, nn=65)
    mdl = nngp_amd.NNGP_p(n=3, N=100, nn=64)
    assert mdl.n_neighbours() == 64
    ad = nngp_amd.NNGP_p(n=3, N=100)
    ad.k = 62
    assert ad.n_neighbours() == 64
    ad.k = 63
    with pytest.raises(ValueError, match='adaptive'):
        ad.n_neighbours()


def test_bench_roofline_traffic_is_the_committed_pmc_figure():
    """bench.py's roofline.traffic comes from the newest committed PMC record (profiles/rNN/
    fine_kernel_traffic.json, tools/pmc_traffic.py): FETCH_SIZE x 2 + WRITE_SIZE, median over the
    headline-length launches, with every launch listed."""
    import json
    import os
    import statistics
    import bench
    tr, src = bench.read_traffic()
    assert tr is not None and src.startswith('profiles/r')
    rec = json.load(open(os.path.join(os.path.dirname(bench.__file__), src)))
    fetch = [d['bytes'] for d in rec['dispatches_fetch_pass'] if d['class'] == 'fine_long']
    write = [d['bytes'] for d in rec['dispatches_write_pass'] if d['class'] == 'fine_long']
    raw = [d['fetch_size_raw_bytes'] for d in rec['dispatches_fetch_pass'] if d['class'] == 'fine_long']
    assert fetch == [2 * r for r in raw]                 # the guide's gfx950 FETCH_SIZE correction
    assert tr['traffic'] == statistics.median(fetch) + statistics.median(write)
    assert len(tr['traffic_all_launches']) == len(fetch)


def test_adaptive_nn_warns_up_front_when_n_could_outgrow_the_fits(monkeypatch):
    """nn='adaptive' (m = k+2) past 63 iterations exceeds the GPU fits' m <= 64: Parareal.run says
    so before any work (the run itself raises only if it gets there)."""
    import warnings
    import nngp_amd as g
    ode = g.Lorenz(normalization='-11')
    s = g.SolverRK(ode.get_vector_field(), Ng=6, Nf=450, F='RK4', G='RK4')
    p = g.Parareal(ode, s, [0, 18], 80, verbose=None)
    monkeypatch.setattr(p, '_parareal', lambda mdl, **kw: {'timings': {}})
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter('always')
        p.run(model='nngp', nn='adaptive')
    assert any('adaptive' in str(x.message) for x in w)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter('always')
        p.run(model='nngp', nn='adaptive', early_stop=40)
    assert not any('adaptive' in str(x.message) for x in w)


@pytest.mark.parametrize('n', [1, 2])
def test_bench_gpus_flag_launches_that_many_ranks(n):
    """`bench.py --gpus N` run bare (no WORLD_SIZE) starts N ranks itself (torch.distributed.run as a
    child process) and its line reports the world the process group saw; --dry-run does the same
    launch on gloo without a GPU.  A world that does not match --gpus exits non-zero."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
    p = subprocess.run([sys.executable, os.path.join(root, 'bench.py'), '--gpus', str(n), '--dry-run'],
                       capture_output=True, text=True, timeout=240, env=env, cwd='/tmp')
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert rec['n_gpus'] == n and rec['ranks_seen'] == list(range(n)) and rec['dry_run']
    # a launcher world that disagrees with --gpus is refused
    bad = subprocess.run([sys.executable, os.path.join(root, 'bench.py'), '--gpus', str(n + 1), '--dry-run'],
                         capture_output=True, text=True, timeout=240, cwd='/tmp',
                         env=dict(env, WORLD_SIZE='1', RANK='0', LOCAL_RANK='0'))
    assert bad.returncode != 0 and 'process group has 1 ranks' in bad.stderr


def test_nngp_training_set_attributes_behave_like_the_reference():
    """NNGP_p.x / .y are plain attributes in the reference (models.py:157-159): readable after
    fit, assignable (the next prediction uses the assigned set), and a clear AttributeError
    before any training set exists."""
    import nngp_amd
    m = nngp_amd.NNGP_p(n=3, N=8, nn=10)
    with pytest.raises(AttributeError, match='fit'):
        m.x
    m.fit(np.zeros((4, 3)), np.ones((4, 3)), k=0)
    assert m.x.shape == (4, 3) and np.all(m.y == 1)
    m.x = np.full((5, 3), 2.0)
    m.y = np.full((5, 3), 3.0)
    assert np.all(m.x == 2) and np.all(m.y == 3) and m._dev_xy is None


def test_published_builders_restate_the_scripts():
    """tests/published_k.py's builders (the published K table's configurations, run by
    tests/test_gpu_published_k.py and bench.py) against the scripts' numbers: steps per slice,
    tspan, u0 and the paged schedule's page arithmetic (tools/paging_delta.py: FHN-PDE d_x = 10
    gets 26 pages, 4 % past the slice end; d_x = 16 and TomLab cover the slice)."""
    import math
    import sys
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    sys.path.insert(0, os.path.join(ROOT, 'tools'))
    import published_k as P
    from paging_delta import pages
    import nngp_amd as g
    want = {   # name: (Nf/N, Ng/N, T0, T1)  -- TomLab.py:72-94, Hopf.py:65-69, FHN_PDE.py:34-57, Burgers.py:27-108
        'tomlab_32_para': (31_250_000, 10, 0, 10), 'tomlab_256_nngp': (3_906_250, 10, 0, 100),
        'tomlab_512_para': (1_953_130, 10, 0, 100), 'hopf_128_nngp': (13_600_000, 16, -20, 500),
        'fhn10_512_nngp': (195_315, 3, 0, 150), 'fhn16_512_nngp': (195_325, 25, 0, 1100),
        'burgers59_128_para': (40_000, 4, 0, 5.9)}
    for name, (nf, ng, a, b) in want.items():
        s, kw, pk = P.build(g, name)
        assert (s.Nf // s.N, s.Ng // s.N) == (nf, ng), name
        assert s.RK_thresh == float('inf') and pk == P.PUBLISHED_K[tuple([name.split('_')[0], int(name.split('_')[1]),
                                                                         name.split('_')[2]])]
        assert float(s.tspan[0]) == a and float(s.tspan[-1]) == b, name
    s, kw, _ = P.build(g, 'tomlab_256_nngp')
    u0 = np.array([4.6722764, 5.2437205e-10, -6.4444208e-10])
    np.testing.assert_array_equal(s.u0, 2 * (u0 + 12) / 24 - 1)   # Systems._tr (new_lib.py:1495-1496)
    assert kw == dict(model='nngp', nn=18, n_restarts=1, fatol=1e-3, xatol=1e-3, seed=45)
    for name, n_pages, cover in (('fhn10_512_nngp_paged', 26, 1.04), ('fhn16_512_nngp_paged', 25, 1.0),
                                 ('tomlab_256_para_paged', 110, 1.0), ('burgers59_128_nngp_paged', 200, 1.0)):
        s, _, _ = P.build(g, name)
        span = (float(s.tspan[-1]) - float(s.tspan[0])) / s.N
        n_p, te = pages(s.Nf // s.N, s.RK_thresh, 0.0, span)
        assert n_p == n_pages and math.isclose(te / span, cover, rel_tol=1e-9), (name, n_p, te / span)
