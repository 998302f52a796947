"""Per-step time of the ODE fine sweep: lane kernel (one slice per lane) vs lane-group kernel
(one slice per 4/16-lane group, components across lanes), same inputs, bitwise compared.

    python tools/lane_group_probe.py [steps_per_slice]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nngp_amd  # noqa: E402


def run(ode, n, steps, quad):
    os.environ['NNGP_RK_GROUP'] = str(quad)
    s = nngp_amd.SolverRK(ode.get_vector_field(), Ng=4, Nf=steps, F='RK4', G='RK1')
    rng = np.random.default_rng(0)
    dev = lambda a: torch.tensor(a, dtype=torch.float64, device='cuda')
    U0 = dev(rng.uniform(-0.5, 0.5, (n, len(ode.get_init_cond()))))
    T0 = dev(np.linspace(0, 1, n))
    T1 = T0 + 1e-3
    s.run_F_batch(T0, T1, U0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    out = s.run_F_batch(T0, T1, U0)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / steps, out.cpu().numpy()


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 400_000
    torch.cuda.set_device(0)
    for name, ode, ns in [('hopf', nngp_amd.Hopf(normalization='-11'), (128, 1024)),
                          ('lorenz', nngp_amd.Lorenz(normalization='-11'), (32, 128)),
                          ('tomlab', nngp_amd.ThomasLabyrinth(normalization='-11'), (32, 256)),
                          ('rossler', nngp_amd.Rossler(normalization='-11'), (128,)),
                          ('fhn_ode', nngp_amd.FHN_ODE(normalization='-11'), (128,)),
                          ('brus', nngp_amd.Brusselator(normalization='-11'), (128,)),
                          ('dblpend', nngp_amd.DblPend(normalization='-11'), (128,))]:
        for n in ns:
            tl, a = run(ode, n, steps, 0)
            tg, b = run(ode, n, steps, 1)
            print(f'{name:8s} n={n:5d} RK4: lane {tl:.4f} us/step  group {tg:.4f} us/step  '
                  f'x{tl / tg:.2f}  bitwise={np.array_equal(a, b)}', flush=True)


if __name__ == '__main__':
    main()
