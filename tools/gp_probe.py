"""GPU probe: full-data GParareal (model='gpjax') on Lorenz N=32 (BASELINE configs[0])."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nngp_amd as g  # noqa: E402

torch.cuda.set_device(0)
ode = g.Lorenz(normalization='-11')
s = g.SolverRK(ode.get_vector_field(), Ng=6, Nf=450, F='RK4', G='RK4')
p = g.Parareal(ode, s, [0, 18], 32, epsilon=5e-7, verbose=None)
t0 = time.perf_counter()
r = p.run(model='gpjax', add_model=True)
dt = time.perf_counter() - t0
m = r['mdl']
print(f"GParareal Lorenz N=32: {dt:.3f} s  K={r['k']}  mdl={r['timings']['mdl_tot_t']:.3f} "
      f"rows={r['x'].shape[0]} rounds={m.rounds} fit_s={np.round(m.tot_train_t[:r['k']], 3).tolist()}",
      flush=True)
