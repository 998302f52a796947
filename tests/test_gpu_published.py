"""Published-scale parity: the legacy new_lib driver surface (nngp_amd.legacy)
runs the reference's own scalability scripts' configurations, with the paging quirk, and must
converge in the published K.  Each run takes minutes of GPU time (Burgers: 200 pages x 39 999
RK8 steps per slice per iteration), so the module runs only with NNGP_PUBLISHED=1:

    NNGP_PUBLISHED=1 python -m pytest tests/test_gpu_published.py -m gpu -v -s --timeout 900
"""
import os

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.slow,
              pytest.mark.skipif(os.environ.get('NNGP_PUBLISHED') != '1', reason='set NNGP_PUBLISHED=1')]


def _burgers(gpu):
    """Burgers.py:27-110 (T=5, the Burges_scal_final_5_128_* runs): N=128, d=128, Ng=4N RK1,
    Nf=Ng*10^4 RK8 (total steps), u0 = 0.5(cos(4.5 pi x)+1) in the '-11' normalisation with bounds
    [0, 1], epsilon 5e-7, RK_thresh = Nf/N/200 (200 pages of 39 999 steps per slice)."""
    N = 128
    ode = gpu.Burgers(d_x=128, normalization='-11')
    s = gpu.legacy.Parareal(f=ode.get_vector_field(), tspan=[0, 5], u0=ode.get_init_cond(), N=N, Ng=N * 4,
                            Nf=N * 4 * 10000, epsilon=5e-7, F='RK8', G='RK1', ode_name='Burg', verbose=None)
    s.RK_thresh = s.Nf / s.N / 200
    return s


def test_burgers_published_schedule_parareal_k(gpu):
    """Burgers d=128 N=128 T=5 on the published schedule -- classic Parareal K=10
    (deterministic: no model randomness, so the published K is asserted exactly)."""
    r = _burgers(gpu).run()
    tm = r['timings']
    print(f"Burgers published schedule parareal: K={r['k']} (published 10) conv_int={r['conv_int']} "
          f"runtime={tm['runtime']:.1f}s F={tm['F_time']:.1f}s")
    assert r['converged'] and r['k'] == 10


@pytest.mark.parametrize('seed', [45, 0, 1, 2])
def test_burgers_published_schedule_nngp_k(gpu, seed):
    """nnGParareal (nn=18, Burgers.py:119; the reference's default seed is 45) on the
    published schedule -- the reference's one published run converged in K=9.  nnGParareal's K
    moves with the Nelder-Mead paths, which move with the seed and with last-ulp differences
    between XLA/LAPACK and this repo's fully specified exp/Cholesky order (the reference's own 100
    seeds at the Burgers_perf_across_m schedule spread over K in {9, 10}); the loop itself is
    pinned bit for bit to the oracle (test_gpu_parareal.py).  Measured on the box
    (profiles/r02/published_nngp_seeds.txt): seeds 45 / 0 / 1 / 2 -> K = 8 / 9 / 10 / 9.
    Asserted: converged within one iteration of the published K."""
    r = _burgers(gpu).run(model='nngp', nn=18, seed=seed)
    tm = r['timings']
    print(f"Burgers published schedule nngp seed {seed}: K={r['k']} (published 9) conv_int={r['conv_int']} "
          f"runtime={tm['runtime']:.1f}s F={tm['F_time']:.1f}s mdl={tm['mdl_tot_t']:.2f}s")
    assert r['converged'] and 8 <= r['k'] <= 10


def test_fhn_pde_d512_published_k(gpu):
    """FHN_PDE.py:27-181 at d_x = 16 (d = 512), N = 512, T = 1100, G = RK4 25 steps/slice, F = RK8
    with the 1e8 schedule (195 325 steps/slice; unpaged here -- the published run paged it, which
    only re-runs the same accurate integration), nnGParareal m = 20: the published run
    (FHN_scal_times_16_512_nngp) converged in K = 6."""
    ode = gpu.FHN_PDE(d_x=16)
    s = gpu.SolverRK(ode.get_vector_field(), Ng=25, Nf=195325, F='RK8', G='RK4', thresh=float('inf'))
    r = gpu.Parareal(ode, s, [0, 1100], 512, epsilon=5e-7, verbose=None).run(model='nngp', nn=20, seed=45)
    print(f"FHN-PDE d=512 N=512: K={r['k']} (published 6) conv_int={r['conv_int']} "
          f"runtime={r['timings']['runtime']:.1f}s")
    assert r['converged'] and r['k'] == 6
