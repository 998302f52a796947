"""GPU probe: full-data GParareal (model='gpjax', models.py:273-473) at BASELINE scale -- Burgers
d=128 N=128 T=5 (Burgers_perf_across_m.py:30-33's 2 000-step schedule, or Burgers.py's published
paged schedule with `pub`): K, conv_int, training rows per iteration, Nelder-Mead rounds, and the
F / model time split.  The published GParareal run (Burges_scal_final_5_128_gp) converged in K = 6.

    python tools/gp_burgers_probe.py [pub] [early_stop]
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nngp_amd as g  # noqa: E402

if __name__ == '__main__':
    torch.cuda.set_device(0)
    pub = 'pub' in sys.argv[1:]
    es = [int(a) for a in sys.argv[1:] if a.isdigit()]
    es = es[0] if es else None
    ode = g.Burgers(d_x=128, normalization='-11')
    if pub:   # Burgers.py:27-110: legacy driver, 200 pages of 39 999 RK8 steps per slice
        N = 128
        p = g.legacy.Parareal(f=ode.get_vector_field(), tspan=[0, 5], u0=ode.get_init_cond(), N=N, Ng=N * 4,
                              Nf=N * 4 * 10000, epsilon=5e-7, F='RK8', G='RK1', ode_name='Burg', verbose=None)
        p.RK_thresh = p.Nf / p.N / 200
    else:
        s = g.SolverRK(ode.get_vector_field(), Ng=4, Nf=2000, F='RK8', G='RK1')
        p = g.Parareal(ode, s, [0, 5], 128, epsilon=5e-7, verbose=None)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = p.run(model='gpjax', early_stop=es, add_model=True)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    tm = r['timings']
    mx = [float(np.nanmax(r['err'][:, k])) for k in range(r['k'])]
    print(f"Burgers N=128 GParareal ({'published schedule' if pub else '2000-step schedule'}): K={r['k']} "
          f"converged={r['converged']} conv_int={r['conv_int']} wall={wall:.2f}s F={tm['F_time']:.2f}s "
          f"G={tm['G_time']:.2f}s mdl={tm['mdl_tot_t']:.2f}s (train {tm['mdl_train_t']:.2f}s, pred {tm['mdl_pred_t']:.2f}s) "
          f"rows={r['x'].shape[0]}", flush=True)
    print('per-iteration max err', [f'{v:.3g}' for v in mx], flush=True)
    mdl = r.get('mdl')
    if mdl is not None:
        print('Nelder-Mead rounds per training call', mdl.rounds, 'fits per call', 128 * 9,
              'training seconds per iteration', [round(float(v), 3) for v in mdl.tot_train_t[:r['k']]], flush=True)
