"""GPU probe: Nelder-Mead evaluation counts of the real Burgers N=128 corrections (iteration 1):
per correction the mean and max nfev over its 1 152 fits, and the kernel time -- the slowest fit
decides the correction's latency."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nngp_amd as g  # noqa: E402

if __name__ == '__main__':
    torch.cuda.set_device(0)
    ode = g.Burgers(d_x=128, normalization='-11')
    s = g.SolverRK(ode.get_vector_field(), Ng=4, Nf=2000, F='RK8', G='RK1')
    r = g.Parareal(ode, s, [0, 5], 128, epsilon=5e-7, verbose=None).run(model='nngp', nn=15, seed=45,
                                                                        early_stop=2)
    dev = lambda a: torch.tensor(np.ascontiguousarray(a), dtype=torch.float64, device='cuda')
    X, Y = dev(r['x']), dev(r['D'])
    mdl = g.NNGP_p(n=128, N=128, nn=15, seed=45)
    fits = torch.empty((mdl.n_fits, 4), dtype=torch.float64, device='cuda')
    means, maxs, ms = [], [], []
    for i in range(1, 128, 8):
        th = dev(mdl.draw_thetas(1))
        q = dev(r['u'][i, :, 1])
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        mdl.predict_device(X, Y, X.shape[0], q, th, fits_out=fits)
        b.record()
        torch.cuda.synchronize()
        F = fits.cpu().numpy()
        nf = F[:, 3]
        slow = F[nf >= 200]
        if len(slow):
            print('   slow fits (theta_x, theta_y, fval, nfev):', np.round(slow[:4], 3).tolist(), flush=True)
        means.append(nf.mean()); maxs.append(nf.max()); ms.append(a.elapsed_time(b))
        print(f'slice {i:3d}: nfev mean {nf.mean():6.1f} p99 {np.percentile(nf, 99):6.1f} max {nf.max():5.0f} '
              f'(#400: {(nf >= 400).sum():3d})  {ms[-1]:.3f} ms', flush=True)
    print(f'avg: nfev mean {np.mean(means):.1f}, max {np.mean(maxs):.1f}, {np.mean(ms):.3f} ms/correction, '
          f'{np.mean(ms) * 1e3 / np.mean(maxs):.2f} us per slowest-fit evaluation')
