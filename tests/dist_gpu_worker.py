"""One rank of tests/test_gpu_distributed.py: a gloo process group over ranks that share the
box's GPU, each running the HIP path of an nnGParareal solve (the fine sweep sharded into
contiguous slice blocks, optionally the corrections sharded by coordinate); rank 0 writes K,
conv_int and the iterates.  Not a test module (no test_ prefix)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def run_case(g, case, shard, native=None):
    """The solves compared across world sizes (same call on 1 rank and on N).  native: the
    library's RCCL communicator for the collectives (run(..., native_comm=...))"""
    if case == 'burgers':   # Burgers_perf_across_m.py's slice schedule on a quarter of the span
        ode = g.Burgers(d_x=128, normalization='-11')
        s = g.SolverRK(ode.get_vector_field(), Ng=4, Nf=2000, F='RK8', G='RK1')
        p = g.Parareal(ode, s, [0, 1.25], 32, epsilon=5e-7, verbose=None)
        kw = dict(model='nngp', nn=15, seed=45, early_stop=3)
    elif case == 'fhn':     # FHN-PDE d=200: 1 800 fits per prediction, sharded by coordinate
        ode = g.FHN_PDE(d_x=10)
        s = g.SolverRK(ode.get_vector_field(), Ng=5, Nf=100, F='RK8', G='RK4')
        p = g.Parareal(ode, s, [0, 8], 16, epsilon=5e-7, verbose=None)
        kw = dict(model='nngp', nn=20, seed=45, early_stop=2)
    elif case == 'tomlab256':   # BASELINE configs[3]: N=256 (32 slices per rank on 8), configs.py schedule
        from nngp_amd.configs import Config
        ode = g.ThomasLabyrinth(normalization='-11')
        cfg = Config(g.ThomasLabyrinth(normalization='-11'), N=256).get()
        s = g.SolverRK(ode.get_vector_field(), Ng=cfg['Ng'], Nf=cfg['Nf'], F='RK4', G='RK1')
        p = g.Parareal(ode, s, cfg['tspan'], 256, epsilon=5e-7, verbose=None)
        kw = dict(model='nngp', nn=18, n_restarts=1, fatol=1e-3, xatol=1e-3, seed=45, early_stop=2)
    elif case == 'fhn800':      # BASELINE configs[4]: FHN-PDE d=800 N=512 (64 slices, 100 coordinates per rank on 8)
        ode = g.FHN_PDE(d_x=20)
        s = g.SolverRK(ode.get_vector_field(), Ng=50, Nf=195325, F='RK8', G='RK4', thresh=float('inf'))
        p = g.Parareal(ode, s, [0, 1100], 512, epsilon=5e-7, verbose=None)
        kw = dict(model='nngp', nn=20, seed=45, early_stop=1)
    elif case == 'gp_burgers':   # GParareal (full-data GP): its d*9 = 576 fits sharded by coordinate
        ode = g.Burgers(d_x=64, normalization='-11')
        s = g.SolverRK(ode.get_vector_field(), Ng=4, Nf=2000, F='RK8', G='RK1')
        p = g.Parareal(ode, s, [0, 1.25], 16, epsilon=5e-7, verbose=None)
        kw = dict(model='gpjax', early_stop=3)
    else:                   # classic Parareal on Lorenz (BASELINE configs[0]'s schedule)
        ode = g.Lorenz(normalization='-11')
        s = g.SolverRK(ode.get_vector_field(), Ng=6, Nf=450, F='RK4', G='RK4')
        p = g.Parareal(ode, s, [0, 18], 32, epsilon=5e-7, verbose=None)
        kw = dict(model='parareal')
    if shard is not None:
        kw['shard_corrections'] = shard
    if native is not None:
        kw['native_comm'] = native
    r = p.run(**kw)
    return r['k'], np.array(r['conv_int']), r['u']


def main():
    case, out, shard = sys.argv[1], sys.argv[2], sys.argv[3]
    shard = None if shard == 'none' else shard == '1'
    import torch
    torch.cuda.set_device(0)
    torch.distributed.init_process_group('gloo')   # MASTER_ADDR/PORT, RANK, WORLD_SIZE from the env
    import nngp_amd as g
    k, conv, u = run_case(g, case, shard)
    if torch.distributed.get_rank() == 0:
        np.savez(out, k=k, conv=conv, u=u)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
