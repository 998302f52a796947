"""GPU probe: Thomas labyrinth N=256 nnGParareal on the configs.py schedule (bench.py's
tomlab_n256_configs_schedule_nngp), first iterations: wall-clock, K, speculation hits.
    python tools/tomlab_probe.py [EARLY_STOP] [SPECULATE (-1 auto, 0 off, 1 on)]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nngp_amd as g  # noqa: E402
from nngp_amd.configs import Config  # noqa: E402


def run(early_stop, speculate=-1):
    ode = g.ThomasLabyrinth(normalization='-11')
    cfg = Config(g.ThomasLabyrinth(normalization='-11'), N=256).get()
    sol = g.SolverRK(ode.get_vector_field(), Ng=cfg['Ng'], Nf=cfg['Nf'], F='RK4', G='RK1')
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = g.Parareal(ode, sol, cfg['tspan'], 256, epsilon=5e-7, verbose=None).run(
        model='nngp', nn=18, n_restarts=1, fatol=1e-3, xatol=1e-3, seed=45, early_stop=early_stop, speculate=speculate)
    torch.cuda.synchronize()
    return time.perf_counter() - t0, r


if __name__ == '__main__':
    es = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    sp = int(sys.argv[2]) if len(sys.argv) > 2 else -1
    torch.cuda.set_device(0)
    run(2, sp)
    s, r = run(es, sp)
    tm = r['timings']
    print(f"TomLab N=256 early_stop={es} speculate={sp}: {s:.3f} s K={r['k']} F={tm['F_time']:.3f} G={tm['G_time']:.3f} "
          f"mdl={tm['mdl_tot_t']:.3f} conv_int={r['conv_int']} hits={tm.get('spec_hits')}", flush=True)
