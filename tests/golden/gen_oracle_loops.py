"""Oracle-loop fixtures for the published-scale parity tests (tests/test_gpu_published.py).

Runs the CPU oracle's restatement of the Parareal loop (oracle/oracle.py `parareal`, OpenMP C
kernels) on configurations too long to run on the GPU box inside the test suite, and commits
the results as small fixtures: K, conv_int, the iterates of the first iterations, a SHA-256 of
the whole iterate array and sampled rows.  The reference itself is not needed (or imported)
here; the oracle is pinned to it by tests/test_oracle_golden.py.

    python tests/golden/gen_oracle_loops.py burgers_pub_nngp_s45   # ~30 min on 8 cores
    python tests/golden/gen_oracle_loops.py fhn800_n512_nngp       # ~15 min
    python tests/golden/gen_oracle_loops.py burgers_pub_nngp_s45_sumorder   # K's roundoff sensitivity
    python tests/golden/gen_oracle_loops.py tomlab256_nngp         # TomLab N=256 to convergence
    python tests/golden/gen_oracle_loops.py burgers128_seeds       # BASELINE configs[2], seeds 0-7 + serial fine
    python tests/golden/gen_oracle_loops.py fhn800_fine            # configs[4]'s serial fine solution (~1e8 steps)
    python tests/golden/gen_oracle_loops.py hopf128_13m_nngp       # bench.py's Hopf solve, 13.6e6 RK4 steps/slice
"""
import hashlib
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, 'oracle'))
import oracle as O  # noqa: E402


def u_digest(u):
    """SHA-256 of the iterate array with NaNs canonicalised (the tests hash the GPU's the same way)."""
    a = np.ascontiguousarray(np.nan_to_num(np.asarray(u, dtype=np.float64), nan=7.0))
    return hashlib.sha256(a.tobytes()).hexdigest()


def _progress(tag, t0):
    def cb(k, st):
        print(f'[{tag}] iteration {k + 1}: I={st["I"]} max err={np.nanmax(st["err"][:, -1]):.3e} '
              f'({time.time() - t0:.0f} s)', flush=True)
    return cb


def burgers_pub(model, seed, nn=18):
    """Burgers.py:27-122 (T=5): new_lib.Parareal with N=128, Ng=4N RK1, Nf=Ng*10^4 RK8 (TOTAL
    steps), '-11' with bounds [0, 1], eps 5e-7, RK_thresh = Nf/N/200 -- 200 pages of 39 999 RK8
    steps per slice per iteration, the legacy global coarse grid and linspace grids."""
    N = 128
    so = O.System('burgers', d=128, param=(0.01,), mn=0.0, mx=1.0)
    x = np.linspace(-1, 1, 128)
    u0 = so.fit(0.5 * (np.cos(4.5 * np.pi * x) + 1))
    Ng, Nf = N * 4, N * 4 * 10000
    thresh = Nf / N / 200
    t0 = time.time()
    kw = dict(model=model) if model == 'parareal' else dict(model=model, nn=nn, seed=seed)
    o = O.parareal(so, [0, 5], N, Ng // N, Nf // N, 'RK1', 'RK8', epsilon=5e-7, u0=u0, step_mode=O.STEP_LINSPACE,
                   coarse_grid=True, F_thresh=thresh, on_iter=_progress(f'burgers {model} {seed}', t0), **kw)
    return o, time.time() - t0


def fhn800(model='nngp'):
    """BASELINE configs[4] (d_x = 20, d = 800, N = 512, T = 1100, no normalisation, u0 =
    systems.py:303-312's seeded draw, nnGParareal m = 20, FHN_PDE.py:175) on FHN_PDE.py's 1e8 fine
    schedule (Nf = ceil(1e8/12800)*12800 -> 195 325 RK8 steps per slice, FHN_PDE.py:54) with G =
    RK4 50 steps per slice, run to convergence.  (configs.py:128-139's default branch, G = RK4
    25/slice with F = RK8 25/slice, is unstable at d_x = 20: the oracle, like the reference's loop,
    stops with 'NaN values in initial coarse solve' after the first iteration -- the GPU test
    checks the same failure.)"""
    so = O.System('fhn_pde', nx=20, normalized=False)
    np.random.seed(45)
    u0 = np.random.Generator(np.random.get_bit_generator()).uniform(size=800)
    t0 = time.time()
    o = O.parareal(so, [0, 1100], 512, 50, 195325, 'RK4', 'RK8', epsilon=5e-7, model=model, nn=20, seed=45, u0=u0,
                   on_iter=_progress('fhn800', t0))
    return o, time.time() - t0


def tomlab256():
    """BASELINE configs[3]'s size to convergence: ThomasLabyrinth N=256 on configs.py's schedule
    (T = 100, G = RK1 10 / F = RK4 3 910 steps per slice) with TomLab.py's nnGP settings (nn = 18,
    fatol = xatol = 1e-3, seed 45), '-11' normalisation, u0 as systems.py:253."""
    so = O.System('tomlab')
    t0 = time.time()
    o = O.parareal(so, [0, 100], 256, 10, 3910, 'RK1', 'RK4', epsilon=5e-7, model='nngp', nn=18, seed=45,
                   fatol=1e-3, xatol=1e-3, u0=so.fit([4.6722764, 5.2437205e-10, -6.4444208e-10]),
                   on_iter=None)
    return o, time.time() - t0


def hopf128_13m():
    """bench.py's `hopf_n128_to_convergence` (BASELINE configs[1] at Hopf.py's throughput schedule):
    Hopf N = 128, '-11' normalisation, G = RK1 16 / F = RK4 13 600 000 steps per slice (Nf =
    2048*85*10^4 / 128, unpaged), Hopf.py's nnGP settings (nn = 15, n_restarts = 2, fatol = xatol =
    0.1, seed 45; Hopf.py:65-84), run to convergence; plus the serial fine solution at every slice
    boundary (128 x 13.6e6 RK4 steps one after another) for the final-state error."""
    so = O.System('hopf', param=(500.0,))
    u0 = so.fit([0.1, 0.1, -20])
    nf = 2048 * 85 * 10000 // 128
    t0 = time.time()
    o = O.parareal(so, [-20, 500], 128, 16, nf, 'RK1', 'RK4', epsilon=5e-7, model='nngp', nn=15, n_restarts=2,
                   fatol=0.1, xatol=0.1, seed=45, u0=u0, on_iter=_progress('hopf128 13.6e6', t0))
    sec = time.time() - t0
    t = np.linspace(-20, 500, 129)
    fine = [u0]
    for i in range(128):
        fine.append(so.rk(4, t[i], t[i + 1], nf, fine[-1]))
    return o, np.array(fine), sec


def burgers_fine(so, u0, N=128, Nf=2000, tspan=(0, 5)):
    """The serial fine solution at the slice boundaries (slice by slice, the F propagator of every
    slice applied to the previous slice's end state -- what a converged Parareal run must equal to
    the convergence tolerance): [N+1][d]."""
    t = np.linspace(tspan[0], tspan[1], N + 1)
    fine = [np.asarray(u0, dtype=float)]
    for i in range(N):
        fine.append(so.rk(8, t[i], t[i + 1], Nf, fine[-1]))
    return np.array(fine)


def burgers128_seeds(seeds):
    """BASELINE configs[2] (Burgers_perf_across_m.py:30-33: d = 128, N = 128, T = 5, F = RK8 2 000 /
    G = RK1 4 steps per slice, '-11' with bounds [0, 1], nn = 15) for several seeds: K, conv_int, a
    digest of every iterate, and the serial fine solution at the slice boundaries with each seed's
    final-state error against it."""
    so = O.System('burgers', d=128, param=(0.01,), mn=0.0, mx=1.0)
    x = np.linspace(-1, 1, 128)
    u0 = so.fit(0.5 * (np.cos(4.5 * np.pi * x) + 1))
    fine = burgers_fine(so, u0)
    out = {'seeds': np.array(seeds), 'fine': fine}
    ks, convs, digs, errs, secs = [], [], [], [], []
    for sd in seeds:
        t0 = time.time()
        o = O.parareal(so, [0, 5], 128, 4, 2000, 'RK1', 'RK8', epsilon=5e-7, model='nngp', nn=15, seed=sd, u0=u0)
        ks.append(o['k'])
        convs.append(np.array(o['conv_int'] + [-1] * (128 - len(o['conv_int']))))
        digs.append(u_digest(o['u']))
        errs.append(np.max(np.abs(o['u'][:, :, -1] - fine)))
        secs.append(time.time() - t0)
        print(f'burgers128 seed {sd}: K={o["k"]} conv_int={o["conv_int"]} final err {errs[-1]:.3e} '
              f'({secs[-1]:.0f} s)', flush=True)
    out.update(k=np.array(ks), conv_int=np.array(convs), digest=np.array(digs),
               final_err=np.array(errs), seconds=np.array(secs))
    return out


def fhn800_fine(rows):
    """The serial fine solution of BASELINE configs[4] (fhn800 above) at the slice boundaries
    `rows`: 512 slices x 195 325 RK8 steps one after another (about 1e8 steps, single thread)."""
    so = O.System('fhn_pde', nx=20, normalized=False)
    np.random.seed(45)
    u = np.random.Generator(np.random.get_bit_generator()).uniform(size=800)
    t = np.linspace(0, 1100, 513)
    keep = {0: u.copy()}
    t0 = time.time()
    for i in range(512):
        u = so.rk(8, t[i], t[i + 1], 195325, u)
        if i + 1 in rows:
            keep[i + 1] = u.copy()
        if i % 16 == 15:
            print(f'fhn800 fine: slice {i + 1}/512 ({time.time() - t0:.0f} s)', flush=True)
    return np.array([keep[r] for r in rows]), time.time() - t0


def main(which):
    if which.startswith('burgers_pub') and 'sumorder' in which:
        # roundoff sensitivity of K on the published schedule: the same run with the GP solves and
        # -LML sums in another summation order (oracle orc_set_sum_order; not a parity fixture)
        O.lib().orc_set_sum_order(1)
        o, sec = burgers_pub('nngp', 45)
        np.savez_compressed(os.path.join(HERE, f'{which}.npz'), k=o['k'], conv_int=np.array(o['conv_int']),
                            converged=o['converged'], digest=u_digest(o['u']), seconds=sec, sum_order=1)
    elif which.startswith('burgers_pub'):
        model = 'parareal' if 'para' in which.split('_')[2] else 'nngp'
        seed = int(which.rsplit('_s', 1)[1]) if model == 'nngp' else 0
        o, sec = burgers_pub(model, seed)
        np.savez_compressed(os.path.join(HERE, f'{which}.npz'), k=o['k'], conv_int=np.array(o['conv_int']),
                            converged=o['converged'], u3=o['u'][:, :, :3], digest=u_digest(o['u']),
                            u_last=o['u'][:, :, -1], seconds=sec)
    elif which == 'tomlab256_nngp':
        o, sec = tomlab256()
        np.savez_compressed(os.path.join(HERE, f'{which}.npz'), k=o['k'], conv_int=np.array(o['conv_int']),
                            converged=o['converged'], digest=u_digest(o['u']), u_last=o['u'][:, :, -1], seconds=sec)
    elif which == 'hopf128_13m_nngp':
        o, fine, sec = hopf128_13m()
        err_max = [float(np.nanmax(o['err'][:, k])) for k in range(o['k'])]
        np.savez_compressed(os.path.join(HERE, f'{which}.npz'), k=o['k'], conv_int=np.array(o['conv_int']),
                            converged=o['converged'], digest=u_digest(o['u']), u_last=o['u'][:, :, -1],
                            u3=o['u'][:, :, :3], err_max=np.array(err_max), fine=fine,
                            final_err=float(np.max(np.abs(o['u'][:, :, -1] - fine))), seconds=sec)
    elif which == 'fhn800_n512_nngp':
        o, sec = fhn800()
        rows = np.array([0, 1, 2, 3, 128, 256, 384, 510, 511, 512])
        np.savez_compressed(os.path.join(HERE, f'{which}.npz'), k=o['k'], conv_int=np.array(o['conv_int']),
                            rows=rows, u_rows=o['u'][rows], digest=u_digest(o['u']), seconds=sec)
    elif which == 'burgers128_seeds':
        out = burgers128_seeds(list(range(8)))
        np.savez_compressed(os.path.join(HERE, f'{which}.npz'), **out)
        print(which, 'K', out['k'].tolist(), 'final err', out['final_err'].tolist(), flush=True)
        return
    elif which == 'fhn800_fine':
        rows = np.load(os.path.join(HERE, 'fhn800_n512_nngp.npz'))['rows']
        fine, sec = fhn800_fine(set(int(r) for r in rows))
        np.savez_compressed(os.path.join(HERE, f'{which}.npz'), rows=rows, fine_rows=fine, seconds=sec)
        print(which, f'{sec:.0f} s', flush=True)
        return
    else:
        raise SystemExit(f'unknown case {which}')
    print(which, 'K', o['k'], 'conv_int', o['conv_int'], 'converged', o['converged'], f'{sec:.0f} s', flush=True)


if __name__ == '__main__':
    main(sys.argv[1])
