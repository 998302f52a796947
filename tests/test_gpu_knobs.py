"""Every environment knob the HIP library reads (INTEGRATION.md "Knobs") selects another launch
shape / kernel variant for the SAME arithmetic: each setting must leave a run bitwise unchanged
(iterates, K, conv_int).  One small nnGParareal run per case, with and without the knob.

The knobs are read on every call (csrc/common.h env_int), so monkeypatch toggles them in-process."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(gpu, case):
    if case == 'burgers':     # d = 128 (wave propagator, LDS-staged kNN), 1 152 fits per prediction
        ode = gpu.Burgers(d_x=128, normalization='-11')
        s = gpu.SolverRK(ode.get_vector_field(), Ng=4, Nf=2000, F='RK8', G='RK1')
        p = gpu.Parareal(ode, s, [0, 1.25], 32, epsilon=5e-7, verbose=None)
        kw = dict(model='nngp', nn=15, seed=45, early_stop=3)
    elif case == 'fhn512':    # d = 512 (point-pair propagator, wave-per-pair D2), 4 608 fits (packed + park)
        ode = gpu.FHN_PDE(d_x=16)
        s = gpu.SolverRK(ode.get_vector_field(), Ng=10, Nf=100, F='RK8', G='RK4')
        p = gpu.Parareal(ode, s, [0, 4], 8, epsilon=5e-7, verbose=None)
        kw = dict(model='nngp', nn=20, seed=45, early_stop=2)
    else:                     # Lorenz (group / lane propagators), 27 fits per prediction
        ode = gpu.Lorenz(normalization='-11')
        s = gpu.SolverRK(ode.get_vector_field(), Ng=6, Nf=450, F='RK4', G='RK4')
        p = gpu.Parareal(ode, s, [0, 18], 32, epsilon=5e-7, verbose=None)
        kw = dict(model='nngp', nn=10, seed=47)
    r = p.run(**kw)
    return r['k'], r['conv_int'], np.nan_to_num(r['u'], nan=7.0)


_BASE = {}

KNOBS = [
    ('burgers', 'NNGP_NM_SPEC', '0'), ('burgers', 'NNGP_NM_SPEC', '1'), ('burgers', 'NNGP_NM_REFILL', '0'),
    ('burgers', 'NNGP_NM_JMAJOR', '0'), ('burgers', 'NNGP_SPEC_OVERLAP', '0'), ('burgers', 'NNGP_RESPEC_W', '0'),
    ('burgers', 'NNGP_RESPEC_W', '8'), ('burgers', 'NNGP_SPEC_MAX_FITS', '0'), ('burgers', 'NNGP_BURGERS_LDS', '1'),
    ('burgers', 'NNGP_NM_PARK', '0'), ('burgers', 'NNGP_CHAIN', '1'), ('fhn512', 'NNGP_D2_WAVES', '0'),
    ('fhn512', 'NNGP_FHN_PAIR', '0'), ('fhn512', 'NNGP_NM_PARK', '0'), ('fhn512', 'NNGP_NM_PARK', '20'),
    ('fhn512', 'NNGP_RK_THREADS', '512'), ('lorenz', 'NNGP_RK_GROUP', '0'), ('lorenz', 'NNGP_CHAIN', '1'),
    ('lorenz', 'NNGP_NM_LEVEL2', '0'), ('fhn512', 'NNGP_RESUME_W4', '0'), ('fhn512', 'NNGP_RESUME_W4', '100000'),
    ('fhn512', 'NNGP_RESUME_W2', '0'), ('burgers', 'NNGP_SPEC_WAIT_US', '0'), ('burgers', 'NNGP_GUESS_FUSED', '0'),
    ('lorenz', 'NNGP_GUESS_FUSED', '0'), ('lorenz', 'NNGP_CHAIN_BARRIER_US', '0'),
    ('burgers', 'NNGP_NM_LANES', '0'), ('burgers', 'NNGP_NM_LANES', '1'), ('lorenz', 'NNGP_NM_LANES', '1'),
    ('burgers', 'NNGP_NM_LANES_WG', '64'), ('burgers', 'NNGP_NM_LPF', '1'), ('burgers', 'NNGP_NM_LPF', '4'), ('burgers', 'NNGP_NM_LANES_FILL', '50'),
    ('burgers', 'NNGP_GDIST', '0'), ('burgers', 'NNGP_HIT_MEAN', '0'), ('burgers', 'NNGP_SWEEP_AHEAD', '0'),
    ('burgers', 'NNGP_G_TIME_EVERY', '1'), ('burgers', 'NNGP_SWEEP_STATS', '1'), ('lorenz', 'NNGP_HIT_MEAN', '0'),
    ('burgers', 'NNGP_SEL_PROF', '1'),
]
# knobs whose neutrality needs a setting these runs do not have, tested where they apply:
# NNGP_COMM_TIMEOUT_S (the communicator's deadline: test_gpu_distributed.py
# ::test_comm_init_without_peers_returns_in_bounded_time, a 2-rank init with no peer)
# NNGP_KEY_LDS (selects over more than 4 096 rows: test_gpu_kernels.py
# ::test_knn_streaming_select_vs_oracle runs every case with and without the LDS key cache)
# NNGP_G_SIDE (an unsplit PDE sweep, i.e. without speculation: test_gpu_parareal.py
# ::test_g_side_stream_is_bitwise)
# NNGP_GPF_SLAB_MB / NNGP_GPF_FUSE / NNGP_GPF_ORDER / NNGP_GPF_FMA (the full-GP factorisation, not on the nnGP
# path: test_gpu_gpfull.py::test_gpfull_lml_and_weights_vs_oracle -- the slab bitwise, the two
# orders and FMA each against the oracle to tolerance, as they change the Cholesky's rounding)
COVERED_ELSEWHERE = ['NNGP_COMM_TIMEOUT_S', 'NNGP_KEY_LDS', 'NNGP_G_SIDE', 'NNGP_GPF_SLAB_MB', 'NNGP_GPF_ORDER',
                     'NNGP_GPF_FMA', 'NNGP_GPF_FUSE']


@pytest.mark.parametrize('case,knob,value', KNOBS)
def test_knob_is_bitwise_neutral(gpu, case, knob, value, monkeypatch):
    if case not in _BASE:
        _BASE[case] = _run(gpu, case)
    k0, c0, u0 = _BASE[case]
    monkeypatch.setenv(knob, value)
    if knob == 'NNGP_CHAIN':
        monkeypatch.setenv('NNGP_CHAIN_PROF', '1')   # the chain's per-phase clocks must not change a bit either
    if knob == 'NNGP_CHAIN_BARRIER_US':
        # the chain's grid-barrier timeout at its floor (4 us per G step: 24 us for Lorenz) -- a
        # barrier that times out reruns the sweep on the launch chain, the same bits
        monkeypatch.setenv('NNGP_CHAIN', '1')
    k1, c1, u1 = _run(gpu, case)
    assert (k1, c1) == (k0, c0)
    assert np.array_equal(u1, u0)
