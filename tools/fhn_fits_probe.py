"""GPU probe: the Nelder-Mead evaluation counts of real FHN-PDE d=800 corrections (the training set
and queries of a 1-iteration nnGParareal run, FHN_PDE.py's 1e8 F schedule), i.e. what the tail
hand-off of the packed fits kernel has to finish: how many fits pass the park cap, and how many
run to maxfev.

    python tools/fhn_fits_probe.py [n_queries]
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nngp_amd as g  # noqa: E402

if __name__ == '__main__':
    nq = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    torch.cuda.set_device(0)
    ode = g.FHN_PDE(d_x=20)
    solver = g.SolverRK(ode.get_vector_field(), Ng=50, Nf=195325, F='RK8', G='RK4', thresh=float('inf'))
    r = g.Parareal(ode, solver, [0, 1100], 512, epsilon=5e-7, verbose=None).run(model='nngp', nn=20, seed=45,
                                                                              early_stop=1)
    X, D = r['x'], r['D']
    U = r['u'][:, :, -1]
    dev = lambda a: torch.tensor(np.ascontiguousarray(a), dtype=torch.float64, device='cuda')
    Xd, Dd = dev(X), dev(D)
    mdl = g.NNGP_p(n=ode.d, N=512, nn=20, seed=7)
    fits = torch.empty((mdl.n_fits, 4), dtype=torch.float64, device='cuda')
    allf = []
    for q in np.linspace(1, 510, nq).astype(int):
        th = dev(mdl.draw_thetas(1))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        mdl.predict_device(Xd, Dd, X.shape[0], dev(U[q]), th, fits_out=fits)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        nf = fits[:, 3].cpu().numpy()
        allf.append(nf)
        print(f'slice {q:3d}: {ms:6.2f} ms  nfev mean {nf.mean():5.1f} p90 {np.percentile(nf, 90):4.0f} '
              f'p99 {np.percentile(nf, 99):4.0f} max {nf.max():4.0f}  >70: {(nf > 70).sum():5d}  '
              f'>150: {(nf > 150).sum():4d}  ==400: {(nf >= 400).sum():3d}', flush=True)
    nf = np.concatenate(allf)
    hist = np.histogram(nf, bins=[0, 40, 70, 100, 150, 200, 300, 399, 401])[0]
    print('rows', X.shape[0], 'fits', nf.size, 'histogram [0,40,70,100,150,200,300,399,401):', hist.tolist())
