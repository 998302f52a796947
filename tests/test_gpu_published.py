"""Published-scale parity: the reference's own scalability configurations, on the
legacy new_lib driver surface (nngp_amd.legacy) with the paging quirk where the scripts had it.

* Burgers (Burgers.py:27-122): classic Parareal must converge in the published K = 10
  (deterministic); nnGParareal seed 45 (the reference's default seed) must be bitwise the CPU
  oracle's loop on the same schedule -- every iterate, K and conv_int -- from the fixture
  tests/golden/burgers_pub_nngp_s45.npz (tests/golden/gen_oracle_loops.py, ~30 min on 8 cores).
* FHN-PDE d = 512 N = 512 (FHN_PDE.py:27-181 at d_x = 16): the published K = 6.
* FHN-PDE d = 800 N = 512 (BASELINE configs[4]): nnGParareal to convergence (511 sequential
  corrections of 7 200 fits per iteration) bitwise the oracle's loop (fixture
  tests/golden/fhn800_n512_nngp.npz); configs.py's default branch diverges like the reference.

Each run takes 10-100 s of GPU time.  The K spread over other seeds is an opt-in extra
(NNGP_PUBLISHED=1, ~6 min)."""
import hashlib
import os

import numpy as np
import pytest

from conftest import golden

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


def u_digest(u):
    """gen_oracle_loops.u_digest: SHA-256 of the iterates with NaNs canonicalised."""
    a = np.ascontiguousarray(np.nan_to_num(np.asarray(u, dtype=np.float64), nan=7.0))
    return hashlib.sha256(a.tobytes()).hexdigest()


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


@pytest.mark.timeout(600)
def test_burgers_published_schedule_parareal_k(gpu):
    """Burgers d=128 N=128 T=5 on the published schedule -- classic Parareal K=10
    (deterministic: no model randomness, so the published K is asserted exactly)."""
    r = _burgers(gpu).run()
    tm = r['timings']
    print(f"Burgers published schedule parareal: K={r['k']} (published 10) conv_int={r['conv_int']} "
          f"runtime={tm['runtime']:.1f}s F={tm['F_time']:.1f}s")
    assert r['converged'] and r['k'] == 10


@pytest.mark.timeout(600)
def test_burgers_published_schedule_nngp_s45_bitwise_oracle_loop(gpu):
    """nnGParareal (nn=18, Burgers.py:119; seed 45) on the published schedule, run to convergence:
    the first two iterations (iterate columns 0-2), K, conv_int and the digest of every iterate
    equal the oracle's loop on the same schedule (stencil F, bitwise the dense one).  The
    reference's one published run reported K = 9; the oracle's K is what is asserted (DESIGN.md
    §5 records the comparison)."""
    P = golden('burgers_pub_nngp_s45.npz')
    r = _burgers(gpu).run(model='nngp', nn=18, seed=45)
    tm = r['timings']
    print(f"Burgers published schedule nngp seed 45: K={r['k']} (oracle {int(P['k'])}, published 9) "
          f"conv_int={r['conv_int']} runtime={tm['runtime']:.1f}s F={tm['F_time']:.1f}s mdl={tm['mdl_tot_t']:.2f}s")
    u3 = P['u3']
    assert np.array_equal(np.nan_to_num(r['u'][:, :, :u3.shape[2]], nan=7.0), np.nan_to_num(u3, nan=7.0))
    assert r['k'] == int(P['k']) and r['conv_int'] == list(P['conv_int'])
    assert r['converged'] == bool(P['converged'])
    assert np.array_equal(np.nan_to_num(r['u'][:, :, -1], nan=7.0), np.nan_to_num(P['u_last'], nan=7.0))
    assert u_digest(r['u']) == str(P['digest'])
    # Against the published run itself: its per-iteration maxima over the slices of
    # err = ||u^{k+1} - u^k||_inf (new_lib.py:1038), as VERDICT.md (round 3) quotes them from
    # Burges_scal_final_5_128_nngp (this repo's permitted safe loaders refuse that pickle, DESIGN.md
    # §5).  Iterations 1-7 agree in magnitude (a factor of 2); the published run's iteration-8
    # maximum 7.37e-7 sits above epsilon = 5e-7 and ours below it, which is why the published
    # run needed a 9th iteration and this one stops at K = 8: a threshold straddle.
    published = [0.117, 0.0179, 3.03e-3, 4.99e-4, 4.62e-5, 4.13e-6, 2.39e-6, 7.37e-7, 2.87e-7]
    ours = [float(np.nanmax(r['err'][:, k])) for k in range(r['k'])]
    print('per-iteration max err: ours', [f'{v:.3g}' for v in ours], 'published', published)
    for k in range(7):
        assert 0.5 <= ours[k] / published[k] <= 2.0, (k + 1, ours[k], published[k])
    assert r['k'] == 8 and ours[7] < 5e-7 < published[7]


@pytest.mark.skipif(os.environ.get('NNGP_PUBLISHED') != '1', reason='set NNGP_PUBLISHED=1 (K spread over seeds)')
@pytest.mark.parametrize('seed', [0, 1, 2])
def test_burgers_published_schedule_nngp_k_other_seeds(gpu, seed):
    """The K spread over other seeds (the reference's 100 seeds on the Burgers_perf_across_m
    schedule spread over K in {9, 10}); profiles/r02/published_nngp_seeds.txt: 9 / 10 / 9."""
    r = _burgers(gpu).run(model='nngp', nn=18, seed=seed)
    print(f"Burgers published schedule nngp seed {seed}: K={r['k']} conv_int={r['conv_int']}")
    assert r['converged'] and 8 <= r['k'] <= 10


@pytest.mark.timeout(300)
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
    # the published run's converged-interval sequence (FHN_scal_times_16_512_nngp, as VERDICT.md
    # round 3 quotes it; the pickle itself is refused by the permitted safe loaders)
    assert r['conv_int'] == [1, 2, 3, 4, 7, 512]


def fhn800_n512(gpu, ng=50, nf=195325):
    """BASELINE configs[4]: FHN-PDE d_x = 20 (d = 800), N = 512, T = 1100 (configs.py:128-139's
    default branch), F = RK8 on FHN_PDE.py's 1e8 schedule (195 325 steps per slice,
    FHN_PDE.py:54), G = RK4 50 steps per slice (the branch's 25 diverge at d_x = 20, see below),
    nnGParareal m = 20 (FHN_PDE.py:175)."""
    ode = gpu.FHN_PDE(d_x=20)
    s = gpu.SolverRK(ode.get_vector_field(), Ng=ng, Nf=nf, F='RK8', G='RK4', thresh=float('inf'))
    return gpu.Parareal(ode, s, [0, 1100], 512, epsilon=5e-7, verbose=None)


@pytest.mark.timeout(300)
def test_fhn_pde_d800_n512_nngp_bitwise_oracle_loop(gpu):
    """BASELINE configs[4] end to end, to convergence: every fine solve (195 325 RK8 steps per
    slice), every sequential correction (7 200 fits each), K and conv_int -- every iterate bitwise
    the oracle loop's (SHA-256 of the iterates + sampled rows; tests/golden/fhn800_n512_nngp.npz)."""
    P = golden('fhn800_n512_nngp.npz')
    r = fhn800_n512(gpu).run(model='nngp', nn=20, seed=45)
    tm = r['timings']
    print(f"FHN-PDE d=800 N=512: K={r['k']} (oracle {int(P['k'])}) conv_int={r['conv_int']} "
          f"runtime={tm['runtime']:.2f}s F={tm['F_time']:.2f}s mdl={tm['mdl_tot_t']:.2f}s")
    assert r['k'] == int(P['k']) and r['conv_int'] == list(P['conv_int'])
    rows = P['rows']
    assert np.array_equal(np.nan_to_num(r['u'][rows], nan=7.0), np.nan_to_num(P['u_rows'], nan=7.0))
    assert u_digest(r['u']) == str(P['digest'])


@pytest.mark.timeout(300)
def test_fhn_pde_d800_default_branch_raises_like_the_reference(gpu):
    """configs.py:128-139's default branch as is (G = RK4 25 steps, F = RK8 25 steps per slice) is
    unstable at d_x = 20 (h*lambda of the stiffest diffusion mode outside RK4's stability
    interval): the reference loop's NaN guard (parareal.py:396-397) stops the run after the first
    iteration, and so does the oracle's (tests/golden/gen_oracle_loops.py) -- and so must this."""
    from nngp_amd.configs import Config
    cfg = Config(gpu.FHN_PDE(d_x=20), d_x=20).get()
    assert (cfg['Ng'], cfg['Nf'], cfg['tspan'], cfg['G'], cfg['F']) == (25, 25, [0, 1100], 'RK4', 'RK8')
    with pytest.raises(Exception, match='NaN values in initial coarse solve'):
        fhn800_n512(gpu, cfg['Ng'], cfg['Nf']).run(model='nngp', nn=20, seed=45)


@pytest.mark.timeout(300)
def test_tomlab_n256_nngp_to_convergence_bitwise_oracle_loop(gpu):
    """BASELINE configs[3]'s size to convergence: ThomasLabyrinth N=256 on configs.py's schedule
    (configs.py:50-57: T=100, Ng/N=10 RK1, Nf/N=3 910 RK4) with TomLab.py's nnGP settings (nn=18,
    fatol=xatol=1e-3, seed 45): K = 162 and every iterate of the 162 iterations bitwise the
    oracle loop's (tests/golden/tomlab256_nngp.npz; the published run on the 1e9 schedule: K = 159)."""
    from nngp_amd.configs import Config
    P = golden('tomlab256_nngp.npz')
    ode = gpu.ThomasLabyrinth(normalization='-11')
    cfg = Config(gpu.ThomasLabyrinth(normalization='-11'), N=256).get()
    s = gpu.SolverRK(ode.get_vector_field(), Ng=cfg['Ng'], Nf=cfg['Nf'], F='RK4', G='RK1')
    r = gpu.Parareal(ode, s, cfg['tspan'], 256, epsilon=5e-7, verbose=None).run(
        model='nngp', nn=18, n_restarts=1, fatol=1e-3, xatol=1e-3, seed=45)
    print(f"TomLab N=256 to convergence: K={r['k']} (oracle {int(P['k'])}) runtime={r['timings']['runtime']:.1f}s")
    assert r['k'] == int(P['k']) and r['conv_int'] == list(P['conv_int'])
    assert np.array_equal(np.nan_to_num(r['u'][:, :, -1], nan=7.0), np.nan_to_num(P['u_last'], nan=7.0))
    assert u_digest(r['u']) == str(P['digest'])
