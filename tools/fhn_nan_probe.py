"""GPU probe: where does FHN-PDE N=512 nnGParareal produce its first non-finite state?  Runs the
driver with a sweep hook that, after each correction sweep, finds the first slice whose new iterate
is non-finite and saves that prediction's inputs (training set, query, theta draws) to
gpurun_out/fhn_nan_case.npz for an offline oracle replay.

    python tools/fhn_nan_probe.py d_x Ng_per_slice Nf_per_slice
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nngp_amd as g  # noqa: E402
from nngp_amd.parareal import Parareal  # noqa: E402


class Probe(Parareal):
    def _correction_sweep(self, torch, model, t_dev, I, N, U1, UG1, UF, UG, X, Y, rows, th0, stream):
        out = super()._correction_sweep(torch, model, t_dev, I, N, U1, UG1, UF, UG, X, Y, rows, th0, stream)
        u = U1.cpu().numpy()
        bad = np.where(~np.all(np.isfinite(u), axis=1))[0]
        print(f'sweep I={I} rows={rows} m={model.n_neighbours()} max|u|={np.nanmax(np.abs(u)):.3g} '
              f'first non-finite slice: {bad[:5]}', flush=True)
        if len(bad):
            i = int(bad[0]) - 1    # the slice whose prediction produced it
            j = i - I
            nf = model.n_fits
            np.savez('gpurun_out/fhn_nan_case.npz', X=X[:rows].cpu().numpy(), Y=Y[:rows].cpu().numpy(),
                     q=U1[i].cpu().numpy(), th0=th0[j * nf:(j + 1) * nf].cpu().numpy(), m=model.n_neighbours(),
                     ug=UG1[i + 1].cpu().numpy(), u_next=u[i + 1], slice=i, I=I)
            raise SystemExit(f'saved the prediction of slice {i}')
        return out


if __name__ == '__main__':
    dx, ng, nf = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    torch.cuda.set_device(0)
    os.makedirs('gpurun_out', exist_ok=True)
    ode = g.FHN_PDE(d_x=dx)
    solver = g.SolverRK(ode.get_vector_field(), Ng=ng, Nf=nf, F='RK8', G='RK4', thresh=float('inf'))
    p = Probe(ode, solver, [0, 1100], 512, epsilon=5e-7, verbose=None, speculate=0)
    p.run(model='nngp', nn=20, seed=45, early_stop=8)
