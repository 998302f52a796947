"""GPU end-to-end: the device-resident Parareal driver with the HIP propagator and nnGP correction,
against the reference's own runs (tests/golden/) and the CPU oracle's restatement of the loop.

Parity contract: identical K (and converged-interval sequence) where K is
roundoff-stable; chaotic Lorenz nnGP: K within +-2 of the reference."""
import numpy as np
import pytest

import oracle as O
from conftest import golden

pytestmark = pytest.mark.gpu


def _lorenz(gpu):
    ode = gpu.Lorenz(normalization='-11')
    s = gpu.SolverRK(ode.get_vector_field(), Ng=6, Nf=450, F='RK4', G='RK4')
    return gpu.Parareal(ode, s, [0, 18], 32, epsilon=5e-7, verbose=None)


def test_lorenz_parareal_matches_reference(gpu):
    P = golden('para_lorenz.npz')
    r = _lorenz(gpu).run(model='parareal')
    assert r['k'] == int(P['para__k'])
    assert r['conv_int'] == list(P['para__conv_int'])
    assert np.nanmax(np.abs(r['u'] - P['para__u'])) < 1e-9
    assert r['converged']
    # identical to the oracle's restatement of the loop
    s = O.System('lorenz')
    o = O.parareal(s, [0, 18], 32, 6, 450, 'RK4', 'RK4', model='parareal', u0=s.fit([-15, -15, 20]))
    assert np.array_equal(np.nan_to_num(r['u'], nan=7.0), np.nan_to_num(o['u'], nan=7.0))


def test_lorenz_nngp_k_distribution_matches_reference(gpu):
    """Chaotic Lorenz: a last-ulp difference in the -LML flips Nelder-Mead branches and moves K
    (the reference itself moves 18 -> 17/19 under a 1-ulp perturbation), so K is
    compared as a distribution over the reference's seeds 45-49."""
    P = golden('para_lorenz.npz')
    s = O.System('lorenz')
    ks, ref = [], []
    for seed in (45, 46, 47, 48, 49):
        r = _lorenz(gpu).run(model='nngp', nn=10, seed=seed)
        assert r['converged']
        ks.append(r['k'])
        ref.append(int(P[f'nngp_s{seed}__k']))
        # converged solution vs the serial fine solution at the slice boundaries
        assert np.max(np.abs(r['u'][:, :, -1] - P['fine'])) < 0.1   # chaos amplifies eps = 5e-7
        # every seed is the oracle's loop bit for bit (K, conv_int, iterates); the spread against
        # the reference below is the restatement's fixed summation order, not the kernels
        o = O.parareal(s, [0, 18], 32, 6, 450, 'RK4', 'RK4', model='nngp', nn=10, seed=seed,
                       u0=s.fit([-15, -15, 20]))
        assert r['k'] == o['k'] and r['conv_int'] == o['conv_int']
        assert np.array_equal(np.nan_to_num(r['u'], nan=7.0), np.nan_to_num(o['u'], nan=7.0))
    print('K gpu', ks, 'reference', ref)   # oracle = gpu: [18, 19, 18, 18, 18]; reference [18, 21, 18, 19, 20]
    assert max(abs(a - b) for a, b in zip(ks, ref)) <= 2   # K within +-2 of the reference
    assert abs(np.mean(ks) - np.mean(ref)) <= 1.5
    assert all(k < 32 for k in ks)   # nnGParareal beats plain Parareal (K=21) on average
    assert np.mean(ks) <= 21


@pytest.mark.parametrize('chain', ['0', '1'])
def test_lorenz_nngp_bitwise_equals_oracle_loop(gpu, chain, monkeypatch):
    """GPU kernels and the CPU oracle share every operation order (incl. exp/log/10^x), so even
    the chaotic Lorenz nnGParareal run is reproduced bit for bit -- by the launch chain and by the
    fused persistent chain (NNGP_CHAIN=1, §8f row 2), which must really run."""
    from nngp_amd import _lib
    monkeypatch.setenv('NNGP_CHAIN', chain)
    n0, _ = _lib.chain_stats()
    r = _lorenz(gpu).run(model='nngp', nn=10, seed=45)
    assert (_lib.chain_stats()[0] > n0) == (chain == '1')
    s = O.System('lorenz')
    o = O.parareal(s, [0, 18], 32, 6, 450, 'RK4', 'RK4', model='nngp', nn=10, seed=45, u0=s.fit([-15, -15, 20]))
    assert r['k'] == o['k'] and r['conv_int'] == o['conv_int']
    assert np.array_equal(np.nan_to_num(r['u'], nan=7.0), np.nan_to_num(o['u'], nan=7.0))


def test_fhn_ode_matches_reference(gpu):
    P = golden('para_fhn.npz')
    ode = gpu.FHN_ODE(normalization='-11')
    s = gpu.SolverRK(ode.get_vector_field(), Ng=4, Nf=4000, F='RK4', G='RK2')
    p = gpu.Parareal(ode, s, [0, 40], 40, epsilon=5e-7, verbose=None)
    r = p.run(model='parareal')
    assert r['k'] == int(P['para__k'])
    assert np.nanmax(np.abs(r['u'] - P['para__u'])) < 1e-9
    r = p.run(model='nngp', nn=15, seed=45)
    assert r['k'] == int(P['nngp_s45__k'])
    assert r['conv_int'] == list(P['nngp_s45__conv_int'])
    assert np.max(np.abs(r['u'][:, :, -1] - P['nngp_s45__u'][:, :, -1])) < 5e-7   # eps
    assert np.max(np.abs(r['u'][:, :, -1] - P['fine'])) < 1e-5
    assert set(r['timings']) >= {'F_time', 'G_time', 'mdl_tot_t', 'runtime', 'F_time_serial_avg'}


def test_tomlab_nngp_bitwise_equals_oracle_loop(gpu):
    """ThomasLabyrinth (TomLab.py settings: RK4/RK1, m=18, fatol=xatol=1e-3) on a short span: the
    sin-based field and the m=18 fits (24-row padded kernel) match the oracle's loop bit for bit."""
    ode = gpu.ThomasLabyrinth(normalization='-11')
    s = gpu.SolverRK(ode.get_vector_field(), Ng=10, Nf=200, F='RK4', G='RK1')
    p = gpu.Parareal(ode, s, [0, 10], 16, epsilon=5e-7, verbose=None)
    kw = dict(nn=18, n_restarts=1, fatol=1e-3, xatol=1e-3, seed=45, early_stop=4)
    r = p.run(model='nngp', **kw)
    so = O.System('tomlab')
    o = O.parareal(so, [0, 10], 16, 10, 200, 'RK1', 'RK4', model='nngp', nn=18, seed=45, fatol=1e-3,
                   xatol=1e-3, u0=so.fit([4.6722764, 5.2437205e-10, -6.4444208e-10]), early_stop=4)
    assert r['k'] == o['k'] and r['conv_int'] == o['conv_int']
    assert np.array_equal(np.nan_to_num(r['u'], nan=7.0), np.nan_to_num(o['u'], nan=7.0))


def test_tomlab_n256_nngp_bitwise_equals_oracle_loop(gpu):
    """BASELINE configs[3]'s size: ThomasLabyrinth N=256 on configs.py's schedule for N=256
    (configs.py:50-57: T=100, Ng/N=10 RK1, Nf/N=3 910 RK4) with TomLab.py's nnGP settings (m=18,
    fatol=xatol=1e-3), three iterations: every iterate bitwise the oracle's loop."""
    from nngp_amd.configs import Config
    ode = gpu.ThomasLabyrinth(normalization='-11')
    cfg = Config(gpu.ThomasLabyrinth(normalization='-11'), N=256).get()
    Ng, Nf = cfg['Ng'], cfg['Nf']
    assert (Ng, Nf, cfg['tspan']) == (10, 3910, [0, 100])
    s = gpu.SolverRK(ode.get_vector_field(), Ng=Ng, Nf=Nf, F='RK4', G='RK1')
    p = gpu.Parareal(ode, s, [0, 100], 256, epsilon=5e-7, verbose=None)
    kw = dict(nn=18, n_restarts=1, fatol=1e-3, xatol=1e-3, seed=45, early_stop=3)
    r = p.run(model='nngp', **kw)
    so = O.System('tomlab')
    o = O.parareal(so, [0, 100], 256, Ng, Nf, 'RK1', 'RK4', model='nngp', nn=18, seed=45, fatol=1e-3,
                   xatol=1e-3, u0=so.fit([4.6722764, 5.2437205e-10, -6.4444208e-10]), early_stop=3)
    assert r['k'] == o['k'] and r['conv_int'] == o['conv_int']
    assert np.array_equal(np.nan_to_num(r['u'], nan=7.0), np.nan_to_num(o['u'], nan=7.0))


def test_burgers_n128_first_iteration_bitwise_equals_oracle(gpu):
    """BASELINE configs[2] (Burgers d=128, N=128, RK8 2000/RK1 4 per slice, m=15): the first
    iteration -- 128 fine solves and 127 sequential corrections of 1 152 fits each -- is bitwise
    the oracle's (the bench times the same iteration on the CPU)."""
    ode = gpu.Burgers(d_x=128, normalization='-11')
    s = gpu.SolverRK(ode.get_vector_field(), Ng=4, Nf=2000, F='RK8', G='RK1')
    r = gpu.Parareal(ode, s, [0, 5], 128, epsilon=5e-7, verbose=None).run(model='nngp', nn=15, seed=45,
                                                                          early_stop=1)
    so = O.System('burgers', d=128, param=(0.01,), mn=0.0, mx=1.0)
    x = np.linspace(-1, 1, 128)
    o = O.parareal(so, [0, 5], 128, 4, 2000, 'RK1', 'RK8', model='nngp', nn=15, seed=45,
                   u0=so.fit(0.5 * (np.cos(4.5 * np.pi * x) + 1)), early_stop=1)
    assert np.array_equal(np.nan_to_num(r['u'], nan=7.0), np.nan_to_num(o['u'], nan=7.0))


@pytest.mark.parametrize('window', ['0', '4'])
@pytest.mark.parametrize('case', ['burgers', 'lorenz'])
def test_speculative_sweep_is_bitwise_and_hits(gpu, case, window, monkeypatch):
    """The speculative sweep (every slice's fits batched up front for a Parareal-guessed query,
    reused where the actual ordered kNN list matches; window > 0: after a miss the next slices are
    re-guessed from the actual state on a side stream) changes no bit of the run."""
    monkeypatch.setenv('NNGP_RESPEC_W', window)
    if case == 'burgers':
        ode = gpu.Burgers(d_x=128, normalization='-11')
        s = gpu.SolverRK(ode.get_vector_field(), Ng=4, Nf=2000, F='RK8', G='RK1')
        mk = lambda spec: gpu.Parareal(ode, s, [0, 5], 128, epsilon=5e-7, verbose=None, speculate=spec)
        kw = dict(nn=15, seed=45, early_stop=3)
    else:
        ode = gpu.Lorenz(normalization='-11')
        s = gpu.SolverRK(ode.get_vector_field(), Ng=6, Nf=450, F='RK4', G='RK4')
        mk = lambda spec: gpu.Parareal(ode, s, [0, 18], 32, epsilon=5e-7, verbose=None, speculate=spec)
        kw = dict(nn=10, seed=47)
    a = mk(0).run(model='nngp', **kw)
    b = mk(1).run(model='nngp', **kw)
    assert a['k'] == b['k'] and a['conv_int'] == b['conv_int']
    assert np.array_equal(np.nan_to_num(a['u'], nan=7.0), np.nan_to_num(b['u'], nan=7.0))
    hits = b['timings']['spec_hits']
    print(case, window, 'speculation hits per iteration', hits)
    assert sum(hits) > 0 and a['timings']['spec_hits'] == [0] * len(hits)


@pytest.mark.parametrize('case', ['burgers', 'lorenz'])
def test_sweep_host_path_variants_are_bitwise(gpu, case, monkeypatch):
    """The sweep's host-path shortcuts against the plain launch chain, each on and all together:
    G and the kNN distances as one launch (NNGP_GDIST), a hit's mean finished in its select from
    coordinates prepared after the batch (NNGP_HIT_MEAN), and the look-ahead that queues the next
    slice's head before the host reads a hit code (NNGP_SWEEP_AHEAD; undone on a miss).  Same hits,
    every iterate bitwise.  Lorenz (chaotic) misses most slices, so the undo path runs often."""
    if case == 'burgers':
        ode = gpu.Burgers(d_x=128, normalization='-11')
        s = gpu.SolverRK(ode.get_vector_field(), Ng=4, Nf=2000, F='RK8', G='RK1')
        p = gpu.Parareal(ode, s, [0, 5], 128, epsilon=5e-7, verbose=None, speculate=1)
        kw = dict(nn=15, seed=45)
    else:
        ode = gpu.Lorenz(normalization='-11')
        s = gpu.SolverRK(ode.get_vector_field(), Ng=6, Nf=450, F='RK4', G='RK4')
        p = gpu.Parareal(ode, s, [0, 18], 32, epsilon=5e-7, verbose=None, speculate=1)
        kw = dict(nn=10, seed=47)
    runs = {}
    for name, knobs in (('plain', ('0', '0', '0')), ('gdist', ('1', '0', '0')), ('hitmean', ('0', '1', '0')),
                        ('all', ('1', '1', '1'))):
        for k, v in zip(('NNGP_GDIST', 'NNGP_HIT_MEAN', 'NNGP_SWEEP_AHEAD'), knobs):
            monkeypatch.setenv(k, v)
        runs[name] = p.run(model='nngp', **kw)
    a = runs['plain']
    for name, b in runs.items():
        print(case, name, 'hits', b['timings']['spec_hits'])
        assert a['timings']['spec_hits'] == b['timings']['spec_hits'], name
        assert a['k'] == b['k'] and a['conv_int'] == b['conv_int'], name
        assert np.array_equal(np.nan_to_num(a['u'], nan=7.0), np.nan_to_num(b['u'], nan=7.0)), name


@pytest.mark.parametrize('case', ['fhn512', 'burgers_lds'])
def test_g_side_stream_is_bitwise(gpu, case, monkeypatch):
    """Without speculation a PDE sweep slice's G runs on a side stream beside its kNN and fits, and
    only the mean waits for it (NNGP_G_SIDE=1, the default): every iterate bitwise the plain chain."""
    if case == 'fhn512':   # FHN-PDE d = 512, point-pair G
        ode = gpu.FHN_PDE(d_x=16)
        s = gpu.SolverRK(ode.get_vector_field(), Ng=10, Nf=100, F='RK8', G='RK4')
        p = gpu.Parareal(ode, s, [0, 4], 8, epsilon=5e-7, verbose=None, speculate=0)
        kw = dict(nn=20, seed=45, early_stop=3)
    else:                  # Burgers on the LDS field kernel (no in-kernel G)
        monkeypatch.setenv('NNGP_BURGERS_LDS', '1')
        ode = gpu.Burgers(d_x=128, normalization='-11')
        s = gpu.SolverRK(ode.get_vector_field(), Ng=4, Nf=2000, F='RK8', G='RK1')
        p = gpu.Parareal(ode, s, [0, 1.25], 32, epsilon=5e-7, verbose=None, speculate=0)
        kw = dict(nn=15, seed=45, early_stop=3)
    monkeypatch.setenv('NNGP_G_SIDE', '0')
    a = p.run(model='nngp', **kw)
    monkeypatch.setenv('NNGP_G_SIDE', '1')
    b = p.run(model='nngp', **kw)
    assert a['k'] == b['k'] and a['conv_int'] == b['conv_int']
    assert np.array_equal(np.nan_to_num(a['u'], nan=7.0), np.nan_to_num(b['u'], nan=7.0))


@pytest.mark.parametrize('case', ['burgers', 'hopf', 'tomlab'])
def test_fused_guess_chain_keeps_hits_and_bits(gpu, case, monkeypatch):
    """The speculative sweep's guesses along the coarse chain by one wave (guess_chain_kernel,
    NNGP_GUESS_FUSED=1, default) against the launch loop (G + update per slice): the same guesses bit
    for bit show as the same speculation hits in every iteration, and the run is bitwise unchanged."""
    if case == 'burgers':      # wave form of G (d = 128, RK1, normalised)
        ode = gpu.Burgers(d_x=128, normalization='-11')
        s = gpu.SolverRK(ode.get_vector_field(), Ng=4, Nf=2000, F='RK8', G='RK1')
        p = gpu.Parareal(ode, s, [0, 5], 128, epsilon=5e-7, verbose=None)
        kw = dict(nn=15, seed=45, early_stop=4)
    elif case == 'hopf':       # lane form, the Markstein division (RK4 G)
        ode = gpu.Hopf(normalization='-11')
        s = gpu.SolverRK(ode.get_vector_field(), Ng=16, Nf=1360, F='RK4', G='RK4')
        p = gpu.Parareal(ode, s, [-20, 500], 128, epsilon=5e-7, verbose=None)
        kw = dict(nn=11, seed=45, early_stop=4)
    else:                      # lane form with nn_sin_pi (RK4 G)
        ode = gpu.ThomasLabyrinth(normalization='-11')
        s = gpu.SolverRK(ode.get_vector_field(), Ng=10, Nf=3910, F='RK4', G='RK4')
        p = gpu.Parareal(ode, s, [0, 10], 64, epsilon=5e-7, verbose=None)
        kw = dict(nn=11, seed=45, early_stop=4)
    monkeypatch.setenv('NNGP_GUESS_FUSED', '0')
    a = p.run(model='nngp', **kw)
    monkeypatch.setenv('NNGP_GUESS_FUSED', '1')
    b = p.run(model='nngp', **kw)
    print(case, 'hits launch loop', a['timings']['spec_hits'], 'fused', b['timings']['spec_hits'])
    assert a['timings']['spec_hits'] == b['timings']['spec_hits'] and sum(b['timings']['spec_hits']) > 0
    assert a['k'] == b['k'] and a['conv_int'] == b['conv_int']
    assert np.array_equal(np.nan_to_num(a['u'], nan=7.0), np.nan_to_num(b['u'], nan=7.0))


def test_auto_speculation_pauses_after_a_low_hit_rate(gpu):
    """speculate=-1 (auto): after an iteration whose guesses hit < 5 % of its slices the next 7
    iterations run without speculation, then it is tried again (a chaotic field: TomLab); the run
    is bitwise the unspeculated one."""
    ode = gpu.ThomasLabyrinth(normalization='-11')
    s = gpu.SolverRK(ode.get_vector_field(), Ng=10, Nf=3910, F='RK4', G='RK1')
    p = gpu.Parareal(ode, s, [0, 100], 256, epsilon=5e-7, verbose=None)
    kw = dict(model='nngp', nn=18, n_restarts=1, fatol=1e-3, xatol=1e-3, seed=45, early_stop=10)
    a = p.run(speculate=0, **kw)
    b = p.run(**kw)
    hits = b['timings']['spec_hits']
    print('TomLab N=256 auto speculation hits per iteration', hits)
    assert hits[0] < 0.05 * 255 and hits[1:8] == [0] * 7
    assert a['k'] == b['k'] and a['conv_int'] == b['conv_int']
    assert np.array_equal(np.nan_to_num(a['u'], nan=7.0), np.nan_to_num(b['u'], nan=7.0))


def test_run_kwargs_override_constructor_settings(gpu):
    """run(..., speculate=...) applies to that run only (the constructor's value otherwise)."""
    ode = gpu.Lorenz(normalization='-11')
    s = gpu.SolverRK(ode.get_vector_field(), Ng=6, Nf=450, F='RK4', G='RK4')
    p = gpu.Parareal(ode, s, [0, 18], 32, epsilon=5e-7, verbose=None, speculate=1)
    a = p.run(model='nngp', nn=10, seed=47, early_stop=3, speculate=0)
    b = p.run(model='nngp', nn=10, seed=47, early_stop=3)
    assert a['timings']['spec_hits'] == [0] * a['k'] and sum(b['timings']['spec_hits']) > 0
    assert np.array_equal(np.nan_to_num(a['u'], nan=7.0), np.nan_to_num(b['u'], nan=7.0))


@pytest.mark.parametrize('model', ['nngp', 'parareal', 'gpjax'])
def test_debug_mode_reports_prediction_errors_without_changing_the_run(gpu, model):
    """run(debug=True) (parareal.py:258-262, 353-406, 441-463): the same iterates, plus per
    iteration |F(u_i) - uG_new - prediction| for every slice and the one-step error table."""
    ode = gpu.Lorenz(normalization='-11')
    s = gpu.SolverRK(ode.get_vector_field(), Ng=6, Nf=450, F='RK4', G='RK4')
    kw = dict(nn=10, seed=46) if model == 'nngp' else {}
    a = gpu.Parareal(ode, s, [0, 18], 32, epsilon=5e-7, verbose=None).run(model=model, early_stop=4, **kw)
    b = gpu.Parareal(ode, s, [0, 18], 32, epsilon=5e-7, verbose=None).run(model=model, early_stop=4, debug=True,
                                                                          **kw)
    assert a['debug_dict'] == {}
    assert np.array_equal(np.nan_to_num(a['u'], nan=7.0), np.nan_to_num(b['u'], nan=7.0))
    dd = b['debug_dict']
    assert dd['one_step_error'].shape == (b['k'], 2)
    assert len(dd['all_pred_err']) == b['k']
    I = 1
    for k, pe in enumerate(dd['all_pred_err']):
        assert pe.shape == (32 - I, 3) and np.all(np.isfinite(pe))
        I = b['conv_int'][k] + 1   # the next sweep starts after the next F increment
    assert np.all(dd['one_step_error'][:, 1] == [pe.max() for pe in dd['all_pred_err']])


@pytest.mark.parametrize('model', ['nngp', 'gpjax'])
def test_pararealight_returns_the_newest_iterate(gpu, model):
    """PararealLight (parareal.py:812-1060): the same iteration with only current/next iterates
    kept; its 'u' after 3 iterations is column 3 of a Parareal run's history, bit for bit."""
    ode = gpu.Lorenz(normalization='-11')
    s = gpu.SolverRK(ode.get_vector_field(), Ng=6, Nf=450, F='RK4', G='RK4')
    kw = dict(nn=10, seed=45) if model == 'nngp' else {}
    light = gpu.PararealLight(ode, s, [0, 18], 32, epsilon=5e-7, verbose=None).run(model=model, early_stop=3, **kw)
    full = gpu.Parareal(ode, s, [0, 18], 32, epsilon=5e-7, verbose=None).run(model=model, early_stop=4, **kw)
    assert light['u'].shape == (33, 3) and 'data_x' not in light
    assert np.array_equal(np.nan_to_num(light['u'], nan=7.0), np.nan_to_num(full['u'][:, :, 3], nan=7.0))
    assert light['conv_int'] == full['conv_int'][:3]
    assert np.array_equal(light['x'], full['x'][:light['x'].shape[0]])
    with pytest.raises(NotImplementedError):
        gpu.PararealLight(ode, s, [0, 18], 32, verbose=None).run(model=model, store_int=True, **kw)


@pytest.mark.parametrize('F,chain', [('RK4', '0'), ('RK8', '0'), ('RK4', '1')])
def test_hopf_n128_nngp_bitwise_equals_oracle_loop(gpu, F, chain, monkeypatch):
    """BASELINE configs[1], Hopf N=128 on the configs.py schedule (configs.py:35-46: Ng/N = 16 RK1,
    Nf/N = 1 360; F = RK4 as BASELINE names it, RK8 as configs.py has it) with Hopf.py's nnGP
    settings (nn=15, n_restarts=2, fatol=xatol=0.1, seed 45; Hopf.py:83-84): every iterate, K and
    the converged-interval sequence equal the oracle's loop bit for bit (speculative sweep on;
    chain '1': the fused persistent chain, which must really run)."""
    from nngp_amd import _lib
    monkeypatch.setenv('NNGP_CHAIN', chain)
    n0, _ = _lib.chain_stats()
    ode = gpu.Hopf(normalization='-11')
    s = gpu.SolverRK(ode.get_vector_field(), Ng=16, Nf=1360, F=F, G='RK1')
    kw = dict(nn=15, n_restarts=2, fatol=0.1, xatol=0.1, seed=45)
    r = gpu.Parareal(ode, s, [-20, 500], 128, epsilon=5e-7, verbose=None).run(model='nngp', **kw)
    so = O.System('hopf', param=(500.0,))
    o = O.parareal(so, [-20, 500], 128, 16, 1360, 'RK1', F, model='nngp', u0=so.fit([0.1, 0.1, -20]), **kw)
    print('Hopf N=128', F, 'K', r['k'], 'conv_int', r['conv_int'], 'spec hits', r['timings']['spec_hits'])
    assert r['converged'] and r['k'] == o['k'] and r['conv_int'] == o['conv_int']
    assert np.array_equal(np.nan_to_num(r['u'], nan=7.0), np.nan_to_num(o['u'], nan=7.0))
    assert (_lib.chain_stats()[0] > n0) == (chain == '1')


def _chain_case(gpu, case):
    """(Parareal, run kwargs) for the fused-chain A/B cases: Burgers (wave G, RK1), Lorenz (RK4 G),
    FHN-ODE (RK2 G, d=2), Hopf (RK1, 2 restarts), Burgers without normalisation, the legacy
    linspace-grid Lorenz and double pendulum (d=4, sincos G)."""
    if case == 'burgers':
        ode = gpu.Burgers(d_x=128, normalization='-11')
        s = gpu.SolverRK(ode.get_vector_field(), Ng=4, Nf=2000, F='RK8', G='RK1')
        return gpu.Parareal(ode, s, [0, 5], 128, epsilon=5e-7, verbose=None), dict(nn=15, seed=45, early_stop=3)
    if case == 'burgers_raw':
        ode = gpu.Burgers(d_x=64)
        s = gpu.SolverRK(ode.get_vector_field(), Ng=4, Nf=1000, F='RK4', G='RK2')
        return gpu.Parareal(ode, s, [0, 5], 64, epsilon=5e-7, verbose=None), dict(nn=12, seed=46, early_stop=3)
    if case == 'lorenz':
        ode = gpu.Lorenz(normalization='-11')
        s = gpu.SolverRK(ode.get_vector_field(), Ng=6, Nf=450, F='RK4', G='RK4')
        return gpu.Parareal(ode, s, [0, 18], 32, epsilon=5e-7, verbose=None), dict(nn=10, seed=47)
    if case == 'lorenz_linspace':
        ode = gpu.Lorenz(normalization='-11')
        s = gpu.SolverRK(ode.get_vector_field(), Ng=6, Nf=450, F='RK4', G='RK4', step_mode='linspace')
        return gpu.Parareal(ode, s, [0, 18], 32, epsilon=5e-7, verbose=None), dict(nn=10, seed=45)
    if case == 'fhn_ode':
        ode = gpu.FHN_ODE(normalization='-11')
        s = gpu.SolverRK(ode.get_vector_field(), Ng=4, Nf=4000, F='RK4', G='RK2')
        return gpu.Parareal(ode, s, [0, 40], 40, epsilon=5e-7, verbose=None), dict(nn=15, seed=45)
    if case == 'hopf':
        ode = gpu.Hopf(normalization='-11')
        s = gpu.SolverRK(ode.get_vector_field(), Ng=16, Nf=1360, F='RK4', G='RK1')
        return (gpu.Parareal(ode, s, [-20, 500], 64, epsilon=5e-7, verbose=None),
                dict(nn=15, n_restarts=2, fatol=0.1, xatol=0.1, seed=45, early_stop=4))
    ode = gpu.DblPend(normalization='-11')
    s = gpu.SolverRK(ode.get_vector_field(), Ng=12, Nf=800, F='RK8', G='RK1')
    return gpu.Parareal(ode, s, [0, 16], 32, epsilon=5e-7, verbose=None), dict(nn=12, seed=45, early_stop=4)


@pytest.mark.parametrize('case', ['burgers', 'burgers_raw', 'lorenz', 'lorenz_linspace', 'fhn_ode', 'hopf',
                                  'dblpend'])
def test_fused_chain_is_bitwise_the_launch_chain(gpu, case, monkeypatch):
    """the runs of speculation hits go through one persistent kernel per run
    (G, kNN, hit check, arg-min, posterior mean and u = pred + uG per slice; the host takes over at
    each miss).  Every iterate, K, conv_int, the hit counts and the G-time key match the unfused
    launch chain (NNGP_CHAIN=0) bit for bit, and the chain really ran."""
    from nngp_amd import _lib
    p, kw = _chain_case(gpu, case)
    monkeypatch.setenv('NNGP_CHAIN', '0')
    n0, s0 = _lib.chain_stats()
    a = p.run(model='nngp', speculate=1, **kw)
    assert _lib.chain_stats() == (n0, s0)
    monkeypatch.setenv('NNGP_CHAIN', '1')
    b = p.run(model='nngp', speculate=1, **kw)
    n1, s1 = _lib.chain_stats()
    print(case, 'K', b['k'], 'hits', b['timings']['spec_hits'], 'chain launches', n1 - n0, 'slices', s1 - s0,
          'G ms', a['timings']['G_time'] * 1e3, b['timings']['G_time'] * 1e3)
    assert a['k'] == b['k'] and a['conv_int'] == b['conv_int']
    assert a['timings']['spec_hits'] == b['timings']['spec_hits']
    assert np.array_equal(np.nan_to_num(a['u'], nan=7.0), np.nan_to_num(b['u'], nan=7.0))
    assert n1 > n0 and s1 - s0 == sum(b['timings']['spec_hits'])
    assert b['timings']['G_time'] > 0


def test_late_overlapped_batch_rerun_is_bitwise(gpu, monkeypatch):
    """The overlapped speculative batch's recovery path: with NNGP_SPEC_WAIT_US=0 a hit slice whose
    batch fits are not finished gives up at once, writes nothing, later hit slices stop waiting,
    and nngp_correction_sweep reruns the sweep with the batch serialised.  The run must be bitwise
    the default one, and the rerun must really have happened."""
    from nngp_amd import _lib
    ode = gpu.Burgers(d_x=128, normalization='-11')
    s = gpu.SolverRK(ode.get_vector_field(), Ng=4, Nf=2000, F='RK8', G='RK1')
    kw = dict(model='nngp', nn=15, seed=45, early_stop=3, speculate=1)
    a = gpu.Parareal(ode, s, [0, 5], 128, epsilon=5e-7, verbose=None).run(**kw)
    n0 = _lib.sweep_late_reruns()
    monkeypatch.setenv('NNGP_SPEC_WAIT_US', '0')
    b = gpu.Parareal(ode, s, [0, 5], 128, epsilon=5e-7, verbose=None).run(**kw)
    late = _lib.sweep_late_reruns() - n0
    print('late reruns', late, 'hits', b['timings']['spec_hits'])
    assert late >= 1
    assert a['k'] == b['k'] and a['conv_int'] == b['conv_int']
    assert a['timings']['spec_hits'] == b['timings']['spec_hits']
    assert np.array_equal(np.nan_to_num(a['u'], nan=7.0), np.nan_to_num(b['u'], nan=7.0))
