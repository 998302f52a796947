"""GPU probe: Burgers N=128 (d=128, m=15) nnGParareal -- first iteration and full run wall-clock."""
import os
import sys
import time

import torch

if os.environ.get('NNGP_PROBE_MAPS'):   # resolve exit-time crash PCs: the process's mappings, written at exit
    import atexit
    atexit.register(lambda: open(os.environ['NNGP_PROBE_MAPS'], 'w').write(open('/proc/self/maps').read()))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nngp_amd as g  # noqa: E402


def run(early_stop=None):
    ode = g.Burgers(d_x=128, normalization='-11')
    solver = g.SolverRK(ode.get_vector_field(), Ng=4, Nf=2000, F='RK8', G='RK1')
    p = g.Parareal(ode, solver, [0, 5], 128, epsilon=5e-7, verbose=None)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if os.environ.get('NNGP_PROBE_STREAM') == '1':   # the run on a non-default stream
        with torch.cuda.stream(torch.cuda.Stream()):
            r = p.run(model='nngp', nn=15, seed=45, early_stop=early_stop)
    else:
        r = p.run(model='nngp', nn=15, seed=45, early_stop=early_stop)
    torch.cuda.synchronize()
    return time.perf_counter() - t0, r


if __name__ == '__main__':
    torch.cuda.set_device(0)
    run(1)
    for es in (1, None):
        s, r = run(es)
        tm = r['timings']
        print(f"early_stop={es}: {s:.3f} s  K={r['k']}  F={tm['F_time']:.3f} G={tm['G_time']:.3f} "
              f"mdl={tm['mdl_tot_t']:.3f} hits={tm.get('spec_hits')}", flush=True)
