"""Per-step time of the fine sweep, exact build vs the opt-in contracted build (SolverRK(fma=True)),
on the published schedules' kernels, with the largest relative end-state difference.

    python tools/contract_probe.py [scale]     # scale multiplies the timed step counts (default 1)
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nngp_amd as g  # noqa: E402


def run(ode, n, steps, tab, mode, fma, span):
    s = g.SolverRK(ode.get_vector_field(), Ng=4, Nf=steps, F=tab, G='RK1', step_mode=mode, fma=fma,
                   thresh=float('inf'))
    d = len(ode.get_init_cond())
    rng = np.random.default_rng(0)
    dev = lambda a: torch.tensor(a, dtype=torch.float64, device='cuda')
    U0 = dev(np.clip(rng.uniform(-0.5, 0.5, (n, d)), -1, 1))
    t = np.linspace(span[0], span[1], n + 1)
    T0, T1 = dev(t[:-1]), dev(t[1:])
    small = g.SolverRK(ode.get_vector_field(), Ng=4, Nf=10, F=tab, G='RK1', step_mode=mode, fma=fma)
    small.run_F_batch(T0, T1, U0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    out = s.run_F_batch(T0, T1, U0)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / steps, out.cpu().numpy()


def main():
    scale = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
    torch.cuda.set_device(0)
    cases = [('tomlab N=256 RK4 linspace', g.ThomasLabyrinth(normalization='-11'), 256, 400_000, 'RK4', 'linspace', (0, 100)),
             ('hopf N=128 RK8 linspace', g.Hopf(normalization='-11'), 128, 200_000, 'RK8', 'linspace', (-20, 500)),
             ('hopf N=128 RK4 fixed', g.Hopf(normalization='-11'), 128, 400_000, 'RK4', 'fixed', (-20, 500)),
             ('lorenz N=32 RK4 fixed', g.Lorenz(normalization='-11'), 32, 400_000, 'RK4', 'fixed', (0, 18)),
             ('burgers d=128 N=128 RK8', g.Burgers(d_x=128, normalization='-11'), 128, 20_000, 'RK8', 'linspace', (0, 5)),
             ('fhn-pde d=800 N=512 RK8', g.FHN_PDE(d_x=20), 512, 1_000, 'RK8', 'fixed', (0, 1100)),
             ('fhn-pde d=800 N=64 RK8', g.FHN_PDE(d_x=20), 64, 2_000, 'RK8', 'fixed', (0, 1100 / 8)),
             ('fhn-pde d=200 N=512 RK8', g.FHN_PDE(d_x=10, normalization='-11'), 512, 4_000, 'RK8', 'linspace', (0, 1100))]
    for name, ode, n, steps, tab, mode, span in cases:
        steps = max(10, int(steps * scale))
        te, a = run(ode, n, steps, tab, mode, False, span)
        tf, b = run(ode, n, steps, tab, mode, True, span)
        rel = max(float(np.max(np.abs(a[i] - b[i])) / max(1.0, float(np.max(np.abs(a[i]))))) for i in range(n))
        print(f'{name:28s} exact {te:8.4f} us/step  contracted {tf:8.4f} us/step  x{te / tf:.3f}  '
              f'max rel diff {rel:.2e}  ({steps} steps)', flush=True)


if __name__ == '__main__':
    main()
