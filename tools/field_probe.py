"""GPU probe: fine-sweep throughput of the PDE field kernel (Burgers d=128 N=128 RK8, FHN-PDE
d=800 N=512 RK8) -- us per RK step and achieved FP64 TFLOP/s (SURVEY.md §8d flop counts)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nngp_amd as g  # noqa: E402

FLOPS = {'burgers': 28160, 'fhn': 215600}


def sweep(name, ode, n, steps, tspan, reps=3):
    solver = g.SolverRK(ode.get_vector_field(), Ng=1, Nf=steps, F='RK8', G='RK1')
    t = np.linspace(tspan[0], tspan[1], n + 1)
    rng = np.random.default_rng(0)
    U = np.clip(ode.get_init_cond()[None, :] + 0.01 * rng.standard_normal((n, ode.d)), -1, 1)
    dev = lambda a: torch.tensor(a, dtype=torch.float64, device='cuda')
    t0, t1, u0 = dev(t[:-1]), dev(t[1:]), dev(U)
    out = torch.empty_like(u0)
    solver.run_F_batch(t0, t1, u0, out=out)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        solver.run_F_batch(t0, t1, u0, out=out)
    b.record()
    torch.cuda.synchronize()
    s = a.elapsed_time(b) / 1e3 / reps
    tf = n * steps * FLOPS[name] / s / 1e12
    print(f'{name:8s} d={ode.d:4d} slices={n:4d} steps={steps:6d}: {s * 1e3:9.2f} ms/sweep  '
          f'{s / steps * 1e6:7.3f} us/step  {n * steps / s:.3e} steps/s  {tf:6.3f} TFLOP/s '
          f'({tf / 78.6 * 100:.2f}% of FP64 VALU peak)', flush=True)


if __name__ == '__main__':
    torch.cuda.set_device(0)
    if len(sys.argv) > 1 and sys.argv[1] == 'fhn':   # FHN-PDE d=800 only (PMC passes: short)
        sweep('fhn', g.FHN_PDE(d_x=20), 512, 500, [0, 1100], reps=1)
        sweep('fhn', g.FHN_PDE(d_x=20), 64, 500, [0, 1100 / 8], reps=1)
        sys.exit(0)
    sweep('burgers', g.Burgers(d_x=128, normalization='-11'), 128, 2000, [0, 5])
    sweep('fhn', g.FHN_PDE(d_x=20), 512, 2000, [0, 1100])
    sweep('fhn', g.FHN_PDE(d_x=20), 64, 2000, [0, 1100 / 8])   # one GPU's share of N=512 on 8 GPUs
