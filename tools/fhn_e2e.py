"""GPU probe: FHN-PDE N=512 nnGParareal (m=20) end to end -- K, wall-clock, F / G / model split.
T = 1100 (FHN_PDE.py d_x=16 / configs.py default branch), F = RK8 with Nf/N fine steps per slice
(FHN_PDE.py's 1e8 schedule: 195 325, unpaged), G = RK4 with Ng/N coarse steps.

    python tools/fhn_e2e.py d_x Ng_per_slice Nf_per_slice [N] [early_stop]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nngp_amd as g  # noqa: E402

if __name__ == '__main__':
    dx, ng, nf = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    N = int(sys.argv[4]) if len(sys.argv) > 4 else 512
    es = int(sys.argv[5]) if len(sys.argv) > 5 else None
    torch.cuda.set_device(0)
    ode = g.FHN_PDE(d_x=dx)
    solver = g.SolverRK(ode.get_vector_field(), Ng=ng, Nf=nf, F='RK8', G='RK4', thresh=float('inf'))
    p = g.Parareal(ode, solver, [0, 1100], N, epsilon=5e-7, verbose='v')
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    try:
        r = p.run(model='nngp', nn=20, seed=45, early_stop=es)
    except Exception as e:   # e.g. the reference's NaN guard on the coarse solve
        print(f'd_x={dx} Ng/N={ng} Nf/N={nf}: FAILED after {time.perf_counter() - t0:.1f}s: {e}', flush=True)
        sys.exit(0)
    torch.cuda.synchronize()
    s = time.perf_counter() - t0
    tm = r['timings']
    print(f"FHN-PDE d={ode.d} N={N} Ng/N={ng} Nf/N={nf}: K={r['k']} converged={r['converged']} wall={s:.2f}s "
          f"F={tm['F_time']:.2f} G={tm['G_time']:.2f} mdl={tm['mdl_tot_t']:.2f} conv_int={r['conv_int']} "
          f"hits={tm.get('spec_hits')}", flush=True)
