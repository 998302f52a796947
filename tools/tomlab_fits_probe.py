"""GPU probe: the fits of one TomLab N=256 correction late in a run (configs schedule, 40
iterations of training data): per-fit evaluation counts and the wall time of one prediction.
    python tools/tomlab_fits_probe.py [ITERATIONS]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nngp_amd as g  # noqa: E402
from nngp_amd.configs import Config  # noqa: E402


def main():
    its = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    torch.cuda.set_device(0)
    ode = g.ThomasLabyrinth(normalization='-11')
    cfg = Config(g.ThomasLabyrinth(normalization='-11'), N=256).get()
    sol = g.SolverRK(ode.get_vector_field(), Ng=cfg['Ng'], Nf=cfg['Nf'], F='RK4', G='RK1')
    r = g.Parareal(ode, sol, cfg['tspan'], 256, epsilon=5e-7, verbose=None).run(
        model='nngp', nn=18, n_restarts=1, fatol=1e-3, xatol=1e-3, seed=45, early_stop=its)
    X, D = r['x'], r['D']
    rows = X.shape[0]
    dev = lambda a: torch.tensor(np.ascontiguousarray(a), dtype=torch.float64, device='cuda')
    Xt, Dt = dev(X), dev(D)
    mdl = g.NNGP_p(n=3, N=256, nn=18, n_restarts=1, seed=45, fatol=1e-3, xatol=1e-3)
    nf = mdl.n_fits
    th0 = dev(mdl.draw_thetas(8))
    fits = torch.empty((nf, 4), dtype=torch.float64, device='cuda')
    q = dev(r['u'][min(its + 5, 255), :, -1])
    mdl.predict_device(Xt, Dt, rows, q, th0[:nf], fits_out=fits)
    torch.cuda.synchronize()
    ts = []
    for j in range(1, 7):
        qj = dev(r['u'][min(its + 5 + 10 * j, 255), :, -1])
        t0 = time.perf_counter()
        mdl.predict_device(Xt, Dt, rows, qj, th0[j * nf:(j + 1) * nf], fits_out=fits)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
        f = fits.cpu().numpy()
        nfev = f[:, 3].astype(int)
        print(f'rows {rows} query {j}: {1e3 * ts[-1]:.3f} ms; nfev max {nfev.max()} mean {nfev.mean():.1f} '
              f'sorted {sorted(nfev.tolist())[-6:]}; +inf fits {int(np.isinf(f[:, 2]).sum())}', flush=True)


if __name__ == '__main__':
    main()
