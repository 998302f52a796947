"""GPU probe: FHN-PDE d=800 nnGParareal (m=20) on N slices for a few iterations -- wall-clock, model
time and speculation hits.  Run once with the default NNGP_SPEC_MAX_FITS and once raised, to see
whether speculating every slice's 7 200 fits pays at this size.

    python tools/fhn_probe.py [N] [iterations]
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nngp_amd as g  # noqa: E402


def run(N, iters):
    ode = g.FHN_PDE(d_x=20)
    solver = g.SolverRK(ode.get_vector_field(), Ng=100, Nf=400, F='RK8', G='RK4')   # 25 RK4 steps (configs.py) diverge at d_x=20
    p = g.Parareal(ode, solver, [0, 1100 * N / 512], N, epsilon=5e-7, verbose=None)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = p.run(model='nngp', nn=20, seed=45, early_stop=iters)
    torch.cuda.synchronize()
    return time.perf_counter() - t0, r


if __name__ == '__main__':
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    torch.cuda.set_device(0)
    s, r = run(N, iters)
    tm = r['timings']
    u = r['u'][:, :, r['k'] - 1] if r['u'].ndim == 3 else r['u']
    print(f"N={N} iters={r['k']}: {s:.3f} s  F={tm['F_time']:.3f} G={tm['G_time']:.3f} "
          f"mdl={tm['mdl_tot_t']:.3f} hits={tm.get('spec_hits')} checksum={float(np.nansum(u)):.17g}",
          flush=True)
