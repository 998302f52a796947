"""How far the published scripts' PAGED fine solve is from the unpaged one, on the CPU
oracle.  The paged solve (RK_last, new_lib.py:57-69) re-uses the slice's full step
count on every page of `thresh` steps' length, i.e. integrates with a `scaling`-times finer step --
AND its page list is `[thresh] * int(t_steps / thresh) + [t_steps % thresh] * (t_steps % thresh != 0)`
in floating point: when t_steps / thresh rounds to exactly `scaling` but the float remainder is
thresh - 1 ulp-ish (not 0), a 26th page follows and F integrates PAST the slice end.  For every
published configuration this prints the page count, the time the pages cover against the slice,
and (for one slice) max |F_paged - F_unpaged| against epsilon = 5e-7.

    python tools/paging_delta.py   # ~5 min on one core
"""
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'oracle'))
import oracle as O  # noqa: E402


def fhn10():
    """FHN_PDE.py:28-57, 146-161 at d_x = 10: Ng = 512*3, Nf = ceil(1e8/Ng)*Ng, T = 150, RK8,
    '-11' with bounds +-1, u0 = seed-45 rand(200), RK_thresh = Nf/N/25."""
    N, Ng = 512, 512 * 3
    Nf = int(math.ceil(1e8 / Ng) * Ng)
    so = O.System('fhn_pde', nx=10, mn=-1.0, mx=1.0)
    np.random.seed(45)
    u0 = so.fit(np.random.Generator(np.random.get_bit_generator()).uniform(size=200))
    t = np.linspace(0, 150, N + 1)
    return so, t, u0, Nf // N, Nf / N / 25


def burgers59():
    """Burgers.py:27-108 (T = 5.9, N = d = 128, Nf = N*4*10^4 RK8, RK_thresh = Nf/N/200)."""
    N = 128
    so = O.System('burgers', d=128, param=(0.01,), mn=0.0, mx=1.0)
    x = np.linspace(-1, 1, 128)
    u0 = so.fit(0.5 * (np.cos(4.5 * np.pi * x) + 1))
    Nf = N * 4 * 10000
    t = np.linspace(0, 5.9, N + 1)
    return so, t, u0, Nf // N, Nf / N / 200


def fhn(d_x):
    """FHN_PDE.py:34-57 settings for d_x in {12, 16} (see fhn10)."""
    mul, T = {12: (12, 550), 16: (25, 1100)}[d_x]
    N, Ng = 512, 512 * mul
    Nf = int(math.ceil(1e8 / Ng) * Ng)
    so = O.System('fhn_pde', nx=d_x, mn=-1.0, mx=1.0)
    np.random.seed(45)
    u0 = so.fit(np.random.Generator(np.random.get_bit_generator()).uniform(size=2 * d_x * d_x))
    t = np.linspace(0, T, N + 1)
    return so, t, u0, Nf // N, Nf / N / 25


def pages(per, thresh, t0, t1):
    """RK_last's page list (new_lib.py:57-69) for t_steps = per + 1 points, and where it ends."""
    pts = int(per)
    iters = [thresh] * int(pts / thresh) + [pts % thresh] * (pts % thresh != 0)
    step = (t1 - t0) / pts
    te = t0
    for temp in iters:
        te = te + step * temp
    return len(iters), te


def main():
    # the page arithmetic of every published schedule (Hopf.py:65-69 / FHN_PDE.py:146-161 /
    # Burgers.py:95-108 / TomLab.py:97-101): Nf / N steps per slice, RK_thresh = Nf / N / scaling
    for name, per, scaling, span, N in (('hopf_32', 2048 * 85 * 10000 // 32, 25, 520, 32),
                                        ('hopf_128', 2048 * 85 * 10000 // 128, 25, 520, 128),
                                        ('hopf_512', 2048 * 85 * 10000 // 512, 25, 520, 512),
                                        ('fhn10', int(math.ceil(1e8 / 1536) * 1536) // 512, 25, 150, 512),
                                        ('fhn12', int(math.ceil(1e8 / 6144) * 6144) // 512, 25, 550, 512),
                                        ('fhn16', int(math.ceil(1e8 / 12800) * 12800) // 512, 25, 1100, 512),
                                        ('burgers', 4 * 10000, 200, 5.9, 128),
                                        ('tomlab_256', 2560 * math.ceil(1e9 / 2560) // 256, 109, 100, 256),
                                        ('tomlab_512', 5120 * math.ceil(1e9 / 5120) // 512, 109, 100, 512)):
        thresh = per / scaling
        n_p, te = pages(per, thresh, 0.0, span / N)
        print(f'{name}: {per} steps per slice, thresh {thresh!r}: {n_p} pages covering {te / (span / N):.6f} of '
              f'the slice', flush=True)
    for name, mk in (('fhn_pde_dx10_n512', fhn10), ('fhn_pde_dx12_n512', lambda: fhn(12)),
                     ('fhn_pde_dx16_n512', lambda: fhn(16)), ('burgers_t5.9_n128', burgers59)):
        so, t, u0, per, thresh = mk()
        U = u0.reshape(1, -1)
        t0 = time.time()
        unp = so.rk_batch(8, t[:1], t[1:2], per, U, O.STEP_LINSPACE, nthreads=1)
        pag = O.legacy_paged_batch(so, 8, t[:1], t[1:2], per, thresh, U, nthreads=1)
        d = float(np.max(np.abs(pag - unp)))
        n_p, te = pages(per, thresh, t[0], t[1])
        print(f'{name}: slice 0, {per} steps unpaged vs {n_p} pages of {per - 1} steps covering '
              f'{(te - t[0]) / (t[1] - t[0]):.6f} of the slice: max |F_paged - F_unpaged| = {d:.3e} = '
              f'{d / 5e-7:.3g} epsilon ({time.time() - t0:.0f} s)', flush=True)


if __name__ == '__main__':
    main()
