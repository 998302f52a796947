"""The non-chaotic half of the parity contract: the same K as the
reference path AND the final state's error against the serial fine solution, for the BASELINE
configurations whose K is roundoff-stable.

* Burgers d=128 N=128 (BASELINE configs[2], Burgers_perf_across_m.py:30-33): seeds 0-7 bitwise the
  oracle loop (K, conv_int, every iterate) and within the config's stated fp64 tolerance 1e-6 of
  the serial fine solution (tests/golden/burgers128_seeds.npz, gen_oracle_loops.py); 100 seeds'
  K distribution against the reference's 100 recorded seeds (Burges_nngp_exp_val_speed, T=5,
  m=15: 68 x K=9, 32 x K=10), each within 1e-6 of the serial fine solution.
  The reference's own per-seed table sits in a pickle that the permitted safe loaders refuse
  (DESIGN.md §5), so the comparison is of distributions over different seeds.
* Hopf N=128 (BASELINE configs[1], configs.py schedule): final state vs the serial fine solution.
* FHN-PDE d=800 N=512 (BASELINE configs[4]): final state vs the serial fine solution at the
  fixture's sampled slice boundaries (tests/golden/fhn800_fine.npz: 512 x 195 325 RK8 steps one
  after another on the CPU oracle).

Errors are in the solver's state units (the '-11' normalised units where the config normalises),
i.e. the units the reference's convergence test err < epsilon = 5e-7 is measured in.  The
reference returns u without its final iterate (parareal.py:469); its last returned column is
what is compared, as the reference's own golden comparisons do."""
import numpy as np
import pytest

import oracle as O
from conftest import golden

pytestmark = pytest.mark.gpu


def _burgers(gpu):
    ode = gpu.Burgers(d_x=128, normalization='-11')
    s = gpu.SolverRK(ode.get_vector_field(), Ng=4, Nf=2000, F='RK8', G='RK1')
    return gpu.Parareal(ode, s, [0, 5], 128, epsilon=5e-7, verbose=None)


def _digest(u):
    import hashlib
    a = np.ascontiguousarray(np.nan_to_num(np.asarray(u, dtype=np.float64), nan=7.0))
    return hashlib.sha256(a.tobytes()).hexdigest()


@pytest.mark.timeout(300)
def test_burgers_n128_seeds_bitwise_oracle_loop_and_final_state(gpu):
    """configs[2] for seeds 0-7: every run equals the oracle loop's bit for bit (K, conv_int, the
    digest of all iterates) and its final state is within 1e-6 of the serial fine solution."""
    P = golden('burgers128_seeds.npz')
    fine = P['fine']
    for j, seed in enumerate(P['seeds']):
        r = _burgers(gpu).run(model='nngp', nn=15, seed=int(seed))
        conv = [int(c) for c in P['conv_int'][j] if c >= 0]
        err = float(np.max(np.abs(r['u'][:, :, -1] - fine)))
        print(f'seed {seed}: K={r["k"]} (oracle {int(P["k"][j])}) final-state error {err:.3e}')
        assert r['converged'] and r['k'] == int(P['k'][j]) and r['conv_int'] == conv
        # against the reference itself: its 100 recorded seeds on this schedule all gave K in
        # {9, 10} (Burges_nngp_exp_val_speed, T = 5, m = 15: 68 x 9, 32 x 10)
        assert r['k'] in (9, 10)
        assert _digest(r['u']) == str(P['digest'][j])
        assert err <= 1e-6   # BASELINE configs[2]: fp64 tol 1e-6


@pytest.mark.slow
@pytest.mark.timeout(600)
def test_burgers_n128_k_distribution_100_seeds(gpu):
    """configs[2] over 100 seeds (0-99): every run converges, within 1e-6 of the serial fine
    solution, in K in {9, 10} as all of the reference's 100 seeds did -- except at most two runs
    at K = 11 (round 4 recorded one of 100: profiles/r04/parity_r4a.txt; a threshold straddle of
    the last unconverged slice, which this test prints) -- and the share of K = 9 is within 0.2 of
    the reference's 68/100 (a two-sample bound: the standard error of the difference of two
    100-run shares at p = 0.68 is 0.066, so 0.2 is three of them)."""
    fine = golden('burgers128_seeds.npz')['fine']
    ks, errs = [], []
    for seed in range(100):
        r = _burgers(gpu).run(model='nngp', nn=15, seed=seed)
        assert r['converged']
        ks.append(r['k'])
        errs.append(float(np.max(np.abs(r['u'][:, :, -1] - fine))))
        if r['k'] not in (9, 10):
            em = [float(np.nanmax(r['err'][:, k])) for k in range(r['k'])]
            print(f'seed {seed}: K={r["k"]} conv_int {r["conv_int"]} per-iteration max err '
                  f'{[f"{v:.3g}" for v in em]} (epsilon 5e-7)')
    hist = {k: ks.count(k) for k in sorted(set(ks))}
    print('K histogram over seeds 0-99:', hist, '(reference, its 100 seeds: {9: 68, 10: 32}); '
          f'final-state error max {max(errs):.3e}, median {np.median(errs):.3e}')
    assert set(ks) <= {9, 10, 11} and ks.count(11) <= 2
    assert abs(ks.count(9) / 100 - 0.68) <= 0.2
    assert max(errs) <= 1e-6


@pytest.mark.parametrize('F', ['RK4', 'RK8'])
def test_hopf_n128_final_state_vs_serial_fine(gpu, F):
    """configs[1] (configs.py schedule: RK1 16 / F 1 360 steps per slice, Hopf.py's nnGP settings):
    nnGParareal converges and its final state is within 1e-5 (20 epsilon) of the serial fine
    solution; the oracle loop gives 5.1e-7 (RK4) and 1.7e-6 (RK8) on this run, which the GPU
    reproduces bit for bit (test_gpu_parareal.py::test_hopf_n128_nngp_bitwise_equals_oracle_loop).
    Classic Parareal (K = 54) within 1e-6."""
    ode = gpu.Hopf(normalization='-11')
    s = gpu.SolverRK(ode.get_vector_field(), Ng=16, Nf=1360, F=F, G='RK1')
    p = gpu.Parareal(ode, s, [-20, 500], 128, epsilon=5e-7, verbose=None)
    so = O.System('hopf', param=(500.0,))
    t = np.linspace(-20, 500, 129)
    fine = [so.fit([0.1, 0.1, -20])]
    for i in range(128):
        fine.append(so.rk(int(F[2]), t[i], t[i + 1], 1360, fine[-1]))
    fine = np.array(fine)
    r = p.run(model='nngp', nn=15, n_restarts=2, fatol=0.1, xatol=0.1, seed=45)
    e = float(np.max(np.abs(r['u'][:, :, -1] - fine)))
    q = p.run(model='parareal')
    ep = float(np.max(np.abs(q['u'][:, :, -1] - fine)))
    print(f'Hopf N=128 {F}: nnGP K={r["k"]} final-state error {e:.3e}; Parareal K={q["k"]} {ep:.3e}')
    assert r['converged'] and e <= 1e-5
    assert q['converged'] and q['k'] == 54 and ep <= 1e-6


@pytest.mark.timeout(300)
def test_fhn_pde_d800_n512_final_state_vs_serial_fine(gpu):
    """configs[4] to convergence (K = 2, bitwise the oracle loop in test_gpu_published.py): the
    final state at the fixture's sampled slice boundaries is within 1e-6 of the serial fine
    solution (512 x 195 325 RK8 steps one after another, tests/golden/fhn800_fine.npz)."""
    from test_gpu_published import fhn800_n512
    P = golden('fhn800_fine.npz')
    r = fhn800_n512(gpu).run(model='nngp', nn=20, seed=45)
    rows = P['rows']
    e = np.max(np.abs(r['u'][rows, :, -1] - P['fine_rows']), axis=1)
    print('FHN-PDE d=800 N=512: K', r['k'], 'final-state error per sampled boundary', dict(zip(rows.tolist(), e)))
    assert r['converged'] and float(e.max()) <= 1e-6


@pytest.mark.timeout(300)
def test_hopf_n128_throughput_schedule_bitwise_oracle_loop_and_final_state(gpu):
    """bench.py's own headline-config solve, `hopf_n128_to_convergence`: BASELINE configs[1] (Hopf
    N = 128, RK1 16 / RK4 13 600 000 steps per slice -- Hopf.py's Nf x 10^4 schedule, unpaged;
    nn = 15, n_restarts = 2, fatol = xatol = 0.1, seed 45; Hopf.py:65-84) to convergence (~40 s).
    K, conv_int, the first three iterates and the SHA-256 of every iterate equal the CPU oracle
    loop's (tests/golden/hopf128_13m_nngp.npz, gen_oracle_loops.py: K = 15, 560 s on 8 cores), and
    the final state is within 1e-6 of the serial fine solution (128 x 13.6e6 RK4 steps one after
    another; the oracle loop's own error is 3.6e-9)."""
    P = golden('hopf128_13m_nngp.npz')
    ode = gpu.Hopf(normalization='-11')
    s = gpu.SolverRK(ode.get_vector_field(), Ng=16, Nf=2048 * 85 * 10000 // 128, F='RK4', G='RK1',
                     thresh=float('inf'))
    r = gpu.Parareal(ode, s, [-20, 500], 128, epsilon=5e-7, verbose=None).run(
        model='nngp', nn=15, n_restarts=2, fatol=0.1, xatol=0.1, seed=45)
    err = float(np.max(np.abs(r['u'][:, :, -1] - P['fine'])))
    print(f"Hopf N=128 13.6e6: K={r['k']} (oracle loop {int(P['k'])}) conv_int {r['conv_int']} "
          f"final-state error {err:.3e} (oracle loop {float(P['final_err']):.3e})")
    assert r['converged'] and r['k'] == int(P['k']) == 15
    assert r['conv_int'] == [int(c) for c in P['conv_int']]
    assert np.array_equal(r['u'][:, :, :3], P['u3'])
    assert _digest(r['u']) == str(P['digest'])
    assert err <= 1e-6
