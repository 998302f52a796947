"""GPU probe: FHN-PDE d = 800 (d_x = 20) point-pair fine sweep, us per RK8 step at 512 and 64
slices (BASELINE configs[4] and one 8-GPU rank's share), alternating an environment knob.

    python tools/fhn_pair_probe.py [KNOB V_A V_B] [steps] [reps]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nngp_amd as g  # noqa: E402


def sweep_us(n_sl, steps, reps):
    ode = g.FHN_PDE(d_x=20)
    s = g.SolverRK(ode.get_vector_field(), Ng=50, Nf=steps, F='RK8', G='RK4', thresh=float('inf'))
    t = np.linspace(0, 1100, 513)
    rng = np.random.default_rng(0)
    U = np.clip(ode.get_init_cond()[None, :] + 0.01 * rng.standard_normal((n_sl, 800)), 0, 1)
    dev = lambda a: torch.tensor(a, dtype=torch.float64, device='cuda')
    t0, t1, u0 = dev(t[:n_sl]), dev(t[1:n_sl + 1]), dev(U)
    out = torch.empty_like(u0)
    s.run_F_batch(t0, t1, u0, out=out)
    best = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        s.run_F_batch(t0, t1, u0, out=out)
        b.record()
        b.synchronize()
        best.append(a.elapsed_time(b) * 1e3 / steps)
    return min(best), float(out.sum().item())


if __name__ == '__main__':
    torch.cuda.set_device(0)
    knob, va, vb = (sys.argv[1:4] if len(sys.argv) > 3 else ('NNGP_FHN_FLAGS', '0', '1'))
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 2000
    reps = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    for n_sl in (512, 64):
        for v in (va, vb, va, vb):
            os.environ[knob] = v
            us, ck = sweep_us(n_sl, steps, reps)
            print(f'{n_sl} slices {knob}={v}: {us:.3f} us/step  checksum {ck:.17g}', flush=True)
