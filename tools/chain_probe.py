"""GPU probe: wall-clock of nnGParareal runs with the fused correction chain (NNGP_CHAIN=1) and with
the launch chain (NNGP_CHAIN=0), bitwise-equal iterates asserted.  Usage: python tools/chain_probe.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nngp_amd as g  # noqa: E402


def cases():
    ode = g.Lorenz(normalization='-11')
    s = g.SolverRK(ode.get_vector_field(), Ng=6, Nf=450, F='RK4', G='RK4')
    yield 'lorenz N=32 m=10', g.Parareal(ode, s, [0, 18], 32, epsilon=5e-7, verbose=None), dict(nn=10, seed=45)
    ode = g.FHN_ODE(normalization='-11')
    s = g.SolverRK(ode.get_vector_field(), Ng=4, Nf=4000, F='RK4', G='RK2')
    yield 'fhn_ode N=40 m=15', g.Parareal(ode, s, [0, 40], 40, epsilon=5e-7, verbose=None), dict(nn=15, seed=45)
    ode = g.Hopf(normalization='-11')
    s = g.SolverRK(ode.get_vector_field(), Ng=16, Nf=1360, F='RK4', G='RK1')
    yield ('hopf N=128 m=15 R=2', g.Parareal(ode, s, [-20, 500], 128, epsilon=5e-7, verbose=None),
           dict(nn=15, n_restarts=2, fatol=0.1, xatol=0.1, seed=45))
    ode = g.Burgers(d_x=128, normalization='-11')
    s = g.SolverRK(ode.get_vector_field(), Ng=4, Nf=2000, F='RK8', G='RK1')
    yield 'burgers N=128 m=15', g.Parareal(ode, s, [0, 5], 128, epsilon=5e-7, verbose=None), dict(nn=15, seed=45)


def timed(p, kw):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = p.run(model='nngp', **kw)
    torch.cuda.synchronize()
    return time.perf_counter() - t0, r


if __name__ == '__main__':
    torch.cuda.set_device(0)
    for name, p, kw in cases():
        res = {}
        for ch in ('0', '1', '0', '1'):
            os.environ['NNGP_CHAIN'] = ch
            t, r = timed(p, kw)
            if ch in res:
                assert np.array_equal(np.nan_to_num(r['u'], nan=7.0), np.nan_to_num(res[ch][1]['u'], nan=7.0))
                res[ch] = (min(t, res[ch][0]), r)
            else:
                res[ch] = (t, r)
        a, b = res['0'][1], res['1'][1]
        assert a['k'] == b['k'] and np.array_equal(np.nan_to_num(a['u'], nan=7.0), np.nan_to_num(b['u'], nan=7.0))
        print(f"{name}: K={b['k']} hits={sum(b['timings']['spec_hits'])} launch chain {res['0'][0]:.4f} s, "
              f"fused chain {res['1'][0]:.4f} s ({res['0'][0] / res['1'][0]:.2f}x)", flush=True)
