"""K of the opt-in contracted propagator (SolverRK(fma=True)) against the exact build, to
convergence, on the Hopf and Thomas-labyrinth configurations whose published-schedule ratios
DESIGN.md quotes (tests/test_gpu_contract.py pins what this prints)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nngp_amd as g  # noqa: E402
from nngp_amd.configs import Config  # noqa: E402


def run(ode, cfg_n, N, F, G, fma, **kw):
    cfg = Config(type(ode)(normalization='-11'), N=cfg_n).get()
    s = g.SolverRK(ode.get_vector_field(), Ng=cfg['Ng'], Nf=cfg['Nf'], F=F, G=G, fma=fma)
    t0 = time.perf_counter()
    r = g.Parareal(ode, s, cfg['tspan'], N, epsilon=5e-7, verbose=None).run(model='nngp', **kw)
    return r['k'], r['converged'], list(r['conv_int']), time.perf_counter() - t0


if __name__ == '__main__':
    torch.cuda.set_device(0)
    cases = [('hopf N=128 configs.py (RK8 1360 / RK1 16), nn=15 R=2', lambda: g.Hopf(normalization='-11'), 128, 128,
              'RK8', 'RK1', dict(nn=15, n_restarts=2, fatol=0.1, xatol=0.1, seed=45)),
             ('tomlab N=32 configs.py (RK4 31250 / RK1 10), nn=18', lambda: g.ThomasLabyrinth(normalization='-11'), 32,
              32, 'RK4', 'RK1', dict(nn=18, fatol=1e-3, xatol=1e-3, seed=45)),
             ('tomlab N=256 configs.py (RK4 3910 / RK1 10), nn=18', lambda: g.ThomasLabyrinth(normalization='-11'), 256,
              256, 'RK4', 'RK1', dict(nn=18, fatol=1e-3, xatol=1e-3, seed=45))]
    for name, mk, cfg_n, N, F, G, kw in cases:
        ke, ce, ie, se = run(mk(), cfg_n, N, F, G, False, **kw)
        kf, cf, i_f, sf = run(mk(), cfg_n, N, F, G, True, **kw)
        print(f'{name}: exact K={ke} converged={ce} ({se:.1f} s) | contracted K={kf} converged={cf} ({sf:.1f} s) '
              f'| conv_int equal: {ie == i_f}', flush=True)
