"""GPU probe: the distribution of Nelder-Mead evaluation counts in Burgers N=128 corrections, and
what predicts a long fit -- its jitter, its coordinate, or the same fit of the slice's previous
query -- for scheduling long fits first in the speculative batch.

For slices 1, 9, ..., 121 it predicts at the slice's iterate-1 and iterate-2 states (the run's final
training set, seed-45 thetas), and prints per query the nfev mean / p50 / p90 / max and the share
at maxfev, per jitter the mean nfev, and the rank correlation of the two queries' nfev vectors."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nngp_amd as g  # noqa: E402


def ranks(v):
    r = np.empty(len(v))
    r[np.argsort(v, kind='stable')] = np.arange(len(v))
    return r


if __name__ == '__main__':
    torch.cuda.set_device(0)
    ode = g.Burgers(d_x=128, normalization='-11')
    s = g.SolverRK(ode.get_vector_field(), Ng=4, Nf=2000, F='RK8', G='RK1')
    r = g.Parareal(ode, s, [0, 5], 128, epsilon=5e-7, verbose=None).run(model='nngp', nn=15, seed=45,
                                                                        early_stop=3)
    dev = lambda a: torch.tensor(np.ascontiguousarray(a), dtype=torch.float64, device='cuda')
    X, Y = dev(r['x']), dev(r['D'])
    mdl = g.NNGP_p(n=128, N=128, nn=15, seed=45)
    fits = torch.empty((mdl.n_fits, 4), dtype=torch.float64, device='cuda')
    th = dev(mdl.draw_thetas(1))
    per_jit = np.zeros(9)
    allv, corr = [], []
    for i in range(1, 128, 8):
        nf = []
        for k in (1, 2):
            mdl.predict_device(X, Y, X.shape[0], dev(r['u'][i, :, k]), th, fits_out=fits)
            nf.append(fits[:, 3].cpu().numpy().copy())
        for k, v in zip((1, 2), nf):
            print(f'slice {i:3d} iterate {k}: nfev mean {v.mean():6.1f} p50 {np.median(v):5.0f} '
                  f'p90 {np.percentile(v, 90):5.0f} max {v.max():4.0f} at maxfev {np.mean(v >= 400):.3f}', flush=True)
            per_jit += v.reshape(128, 9).mean(0)
            allv.append(v)
        corr.append(np.corrcoef(ranks(nf[0]), ranks(nf[1]))[0, 1])
    allv = np.concatenate(allv)
    print('all: mean %.1f p50 %.0f p90 %.0f p99 %.0f max %.0f, sum of top 10%% = %.2f of all evaluations'
          % (allv.mean(), np.median(allv), np.percentile(allv, 90), np.percentile(allv, 99), allv.max(),
             np.sort(allv)[-len(allv) // 10:].sum() / allv.sum()))
    print('mean nfev per jitter index (1e-20 .. 1e-12):', np.round(per_jit / (2 * len(corr)), 1).tolist())
    print('rank correlation of a fit\'s nfev between the slice\'s two queries: mean %.3f' % np.mean(corr))
