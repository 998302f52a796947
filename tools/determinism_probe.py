"""GPU probe: is an nnGParareal run bitwise reproducible?  Runs the same FHN-PDE N=512 solve
several times (speculation auto / off) for a few iterations and prints a checksum of every
iterate plus the first iteration/slice where two runs differ.

    python tools/determinism_probe.py d_x Ng Nf iterations
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nngp_amd as g  # noqa: E402

if __name__ == '__main__':
    dx, ng, nf, it = (int(a) for a in sys.argv[1:5])
    torch.cuda.set_device(0)
    ode = g.FHN_PDE(d_x=dx)
    solver = g.SolverRK(ode.get_vector_field(), Ng=ng, Nf=nf, F='RK8', G='RK4', thresh=float('inf'))
    runs = []
    for spec in (-1, -1, 0):
        p = g.Parareal(ode, solver, [0, 1100], 512, epsilon=5e-7, verbose=None, speculate=spec)
        try:
            r = p.run(model='nngp', nn=20, seed=45, early_stop=it)
            u = np.nan_to_num(r['u'], nan=7.0)
            print(f'speculate={spec}: K={r["k"]} conv_int={r["conv_int"]} checksum={float(np.sum(np.abs(u))):.17g}',
                  flush=True)
            runs.append(u)
        except Exception as e:
            print(f'speculate={spec}: FAILED {e}', flush=True)
            runs.append(None)
    base = runs[0]
    for j, u in enumerate(runs[1:], 1):
        if base is None or u is None or base.shape != u.shape:
            print('run', j, 'not comparable')
            continue
        diff = np.argwhere(base != u)
        if len(diff) == 0:
            print('run', j, 'bitwise equal to run 0')
        else:
            k = diff[:, 2].min()
            sl = diff[diff[:, 2] == k][:, 0].min()
            print('run', j, 'differs first at iteration', k, 'slice', sl, 'count', len(diff))
