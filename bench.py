"""bench.py -- nnGParareal hot path on MI355X.

Metric (BASELINE.json): fine RK steps/sec + nnGP corrections/sec; wall-clock to convergence (K).
Workload at N=1 (BASELINE.json configs[1]): non-autonomous Hopf, N=128 time slices, RK4 fine
solver with Hopf.py's throughput schedule (Nf = 2048*85*10^4 -> 13.6e6 steps per slice, unpaged),
G = RK1 16 steps/slice, nnGP m=15, 2 restarts, fatol = xatol = 0.1, eps = 5e-7 (Hopf.py:65-84).

One timed "step" = one Parareal fine sweep: every slice propagated by the batched HIP RK kernel
(inputs resident in HBM), followed -- for N>1 -- by the single RCCL all-gather of the fine end
states.  Weak scaling: every rank owns 128 slices, so the job integrates 128*N slices per step.
value = (slices x fine steps per slice, all ranks) / max-over-ranks wall time of the K steps.

Also reported (rank 0): nnGP corrections/s (the sequential correction sweep of one iteration on
the same config), wall-clock to convergence with its K for the full nnGParareal solve of the
Hopf config and of the Burgers d=128 N=128 config (BASELINE configs[2], the north star's 10x
target), the FP64-VALU roofline of the fine kernel (HIP events around the launches), and the CPU
baseline: the oracle's C restatement (OpenMP over slices) on a bounded sample of the same sweep.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 vector: half the 157.3 TF FP32 vector peak (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0
# One-wave issue floor of the fine-sweep kernel: a slice is one dependent chain, so
# a step costs (VALU per step) x (cycles per wave64 VALU issue).  The Hopf sweep at 128 slices runs
# the lane-group kernel (components across a 16-lane group): 85 VALU per RK4 step in the gfx950
# code object since round 3's carried bank-masked RHS registers (97 before; tools/isa_loop_count.py
# rk_group_kernelILi1ELi4ELb0ELb1E; the one-lane-per-slice kernel has 119); 4.22 cycles per
# independent v_mul/v_add_f64 and a 2.40 GHz shader clock measured on the box (tools/ubench_fp64.hip).
LANE_VALU_PER_STEP = 85
CYCLES_PER_F64_VALU = 4.22
SHADER_GHZ = 2.40
# algorithmic flops per fine step per slice: S*F_rhs + (2 nnz(a) + S + 2 nnz(b))*d
FLOPS_PER_STEP = {('hopf', 'RK4'): 126, ('hopf', 'RK8'): 11 * 18 + (2 * 39 + 11 + 2 * 5) * 3,
                  ('burgers', 'RK8'): 28160}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def launch_ranks(n, argv):
    """`bench.py --gpus N` without a launcher around it (WORLD_SIZE unset): start N ranks, one per
    GPU, as `python -m torch.distributed.run --nproc-per-node N` -- a CHILD process, started before
    this process touches the GPU (no exec of a GPU-initialised process) -- and exit with its
    status.  The reference's equivalent is the `srun ... mpi4py.futures` launch of Hopf.py:43-46,
    95-140.  Rank 0 prints the JSON line; its stdout is this process's."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={n}',
           '--master-addr', '127.0.0.1', '--master-port', str(port), os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY='0'))


def dist_init(expect_world, dry_run=False):
    """One process per GPU (LOCAL_RANK -> cuda:LOCAL_RANK), RCCL process group for N > 1.  The world
    the process group reports must be the --gpus the run was asked for, and the node must have that
    many devices; otherwise exit non-zero rather than print a line for another configuration.
    dry_run: the same launch and process group on gloo without a GPU (tests/test_host.py)."""
    import torch
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        if dry_run:
            torch.distributed.init_process_group('gloo')
        else:
            ndev = torch.cuda.device_count()
            if ndev < world:
                sys.exit(f'bench.py: world size {world} needs {world} GPUs, this node has {ndev}')
            torch.cuda.set_device(local)
            torch.distributed.init_process_group('nccl', device_id=torch.device('cuda', local))
        world = torch.distributed.get_world_size()
    elif not dry_run:
        torch.cuda.set_device(0)
    if world != expect_world:
        sys.exit(f'bench.py: --gpus {expect_world} but the process group has {world} ranks')
    return world, rank


def barrier_sync(torch, world):
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()


def hopf_setup(g, steps_per_slice, n_slices):
    ode = g.Hopf(normalization='-11')
    solver = g.SolverRK(ode.get_vector_field(), Ng=2048 // 128, Nf=steps_per_slice, F='RK4', G='RK1',
                        thresh=float('inf'))
    return ode, solver


def fine_sweep_bench(torch, g, world, rank, steps, warmup, steps_per_slice, slices_per_rank):
    """Time K fine sweeps of 128*world slices (weak scaling), HIP events around the kernel."""
    n_total = slices_per_rank * world
    ode, solver = hopf_setup(g, steps_per_slice, n_total)
    rng = np.random.default_rng(1234)
    # synthetic initial data: states uniformly inside the normalised box, times along [-20, 500]
    t = np.linspace(-20, 500, n_total + 1)
    U = rng.uniform(-0.5, 0.5, size=(n_total, 3))
    dev = lambda a: torch.tensor(a, dtype=torch.float64, device='cuda')
    lo, hi = rank * slices_per_rank, (rank + 1) * slices_per_rank
    t0, t1, u0 = dev(t[lo:hi]), dev(t[lo + 1:hi + 1]), dev(U[lo:hi])
    out = torch.empty_like(u0)
    gathered = torch.empty((n_total, 3), dtype=torch.float64, device='cuda')
    ev = []
    # the all-gather of the end states: torch.distributed's (RCCL); the library's own communicator
    # (include/nngp.h nngp_allgather_states) is checked against it after the timed region
    st = torch.cuda.current_stream().cuda_stream

    def one(record):
        if record:
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
        solver.run_F_batch(t0, t1, u0, out=out)
        if record:
            b.record()
            ev.append((a, b))
        if world > 1:
            torch.distributed.all_gather_into_tensor(gathered, out)

    for _ in range(warmup):
        one(False)
    barrier_sync(torch, world)
    t_start = time.perf_counter()
    for _ in range(steps):
        one(True)
    barrier_sync(torch, world)
    elapsed = time.perf_counter() - t_start
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device='cuda')
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(tt.item())
    kernel_s = np.mean([a.elapsed_time(b) / 1e3 for a, b in ev])
    check = None
    if world > 1 and not g.parareal.native_comm_default():
        check = {'nngp_allgather_states_bitwise_torch': None,
                 'note': 'library communicator not exercised: opt-in, NNGP_NATIVE_COMM=1'}
    elif world > 1:   # the library's RCCL all-gather on the same end states, bitwise torch's
        try:
            if g._lib.comm_for(None):
                native = torch.full_like(gathered, float('nan'))
                g._lib.check(g.lib().nngp_allgather_states(out.data_ptr(), native.data_ptr(), out.numel(), st))
                torch.cuda.synchronize()
                same = torch.tensor([1 if torch.equal(native, gathered) else 0], dtype=torch.int32, device='cuda')
                torch.distributed.all_reduce(same, op=torch.distributed.ReduceOp.MIN)
                check = {'nngp_allgather_states_bitwise_torch': bool(same.item())}
            else:
                check = {'nngp_allgather_states_bitwise_torch': None, 'note': 'library communicator unavailable'}
        except Exception as e:   # a report, never fatal to the headline
            check = {'nngp_allgather_states_bitwise_torch': None, 'error': str(e)[:200]}
    return elapsed, kernel_s, n_total, out, ('torch all_gather_into_tensor' if world > 1 else None), check


def corrections_bench(torch, g, m=15, R=2, n_slices=128):
    """One iteration's sequential nnGP correction sweep on Hopf-config training data."""
    ode = g.Hopf(normalization='-11')
    solver = g.SolverRK(ode.get_vector_field(), Ng=16, Nf=1360, F='RK4', G='RK1')
    p = g.Parareal(ode, solver, [-20, 500], n_slices, epsilon=5e-7, verbose=None)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = p.run(model='nngp', nn=m, n_restarts=R, fatol=0.1, xatol=0.1, seed=45, early_stop=2)
    torch.cuda.synchronize()
    # predictions per iteration = N - I with I the first unconverged slice after the F sweep
    n_pred = sum(n_slices - i for i in [1] + [c + 1 for c in r['conv_int'][:-1]])
    return n_pred, r['timings']['mdl_pred_t'], time.perf_counter() - t0


def converge(torch, g, which, fma=False):
    if which == 'hopf':
        ode = g.Hopf(normalization='-11')
        solver = g.SolverRK(ode.get_vector_field(), Ng=16, Nf=2048 * 85 * 10000 // 128, F='RK4', G='RK1',
                            thresh=float('inf'), fma=fma)
        p = g.Parareal(ode, solver, [-20, 500], 128, epsilon=5e-7, verbose=None)
        kw = dict(nn=15, n_restarts=2, fatol=0.1, xatol=0.1, seed=45)
    else:   # Burgers_perf_across_m.py:30-33 (d=128, N=128, T=5, Nf/N=2000 RK8, Ng/N=4 RK1), m=15
        ode = g.Burgers(d_x=128, normalization='-11')
        solver = g.SolverRK(ode.get_vector_field(), Ng=4, Nf=2000, F='RK8', G='RK1', fma=fma)
        p = g.Parareal(ode, solver, [0, 5], 128, epsilon=5e-7, verbose=None)
        kw = dict(nn=15, seed=45)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = p.run(model='nngp', **kw)
    torch.cuda.synchronize()
    r['timings']['conv_int'] = list(r['conv_int'])
    return time.perf_counter() - t0, r['k'], r['converged'], r['timings'], r


def published_runs(torch, g):
    """Two whole nnGParareal solves at the reference's scale, each beside the reference's own figure:
    - Burgers, Burgers.py's published schedule (legacy driver, N = 128, 200 pages of 39 999 RK8 steps
      per slice per iteration, nn = 18, seed 45): the reference's published run took 3 789 s
      (Burges_scal_final, 282 cores) and converged in K = 9; this solve is bitwise the oracle loop's
      (K = 8, tests/test_gpu_published.py);
    - ThomasLabyrinth N = 256 on configs.py's schedule (RK4 3 910 / RK1 10 per slice, nn = 18,
      fatol = xatol = 1e-3): K = 162, bitwise the oracle loop's."""
    out = {}
    N = 128
    ode = g.Burgers(d_x=128, normalization='-11')
    s = g.legacy.Parareal(f=ode.get_vector_field(), tspan=[0, 5], u0=ode.get_init_cond(), N=N, Ng=N * 4,
                          Nf=N * 4 * 10000, epsilon=5e-7, F='RK8', G='RK1', ode_name='Burg', verbose=None)
    s.RK_thresh = s.Nf / s.N / 200
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = s.run(model='nngp', nn=18, seed=45)
    torch.cuda.synchronize()
    w = time.perf_counter() - t0
    out['burgers_n128_published_schedule_nngp'] = {
        'wall_s': w, 'K': r['k'], 'converged': r['converged'], 'F_time_s': r['timings']['F_time'],
        'mdl_time_s': r['timings']['mdl_tot_t'], 'reference_wall_s_282_cores': 3789.0, 'reference_K': 9,
        'speedup_vs_reference_wall': 3789.0 / w, 'K_oracle_loop': 8,
        'note': 'K differs from the published 9 by one; the oracle loop gives 8 too (DESIGN.md section 5)'}
    from nngp_amd.configs import Config
    ode = g.ThomasLabyrinth(normalization='-11')
    cfg = Config(g.ThomasLabyrinth(normalization='-11'), N=256).get()
    sol = g.SolverRK(ode.get_vector_field(), Ng=cfg['Ng'], Nf=cfg['Nf'], F='RK4', G='RK1')
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = g.Parareal(ode, sol, cfg['tspan'], 256, epsilon=5e-7, verbose=None).run(
        model='nngp', nn=18, n_restarts=1, fatol=1e-3, xatol=1e-3, seed=45)
    torch.cuda.synchronize()
    out['tomlab_n256_configs_schedule_nngp'] = {
        'wall_s': time.perf_counter() - t0, 'K': r['k'], 'converged': r['converged'],
        'F_time_s': r['timings']['F_time'], 'mdl_time_s': r['timings']['mdl_tot_t'], 'K_oracle_loop': 162,
        'schedule': 'configs.py N=256 (RK4 3910 / RK1 10 per slice); the published run used the 1e9 schedule (K=159)'}
    return out


def published_k_table(torch, g, live_extra=None):
    """The reference's published K table (tests/published_k.py: Hopf.py, FHN_PDE.py, Burgers.py on
    the legacy driver).  Run live here: Burgers T = 5.9 and FHN-PDE d_x = 10 classic Parareal (~25 s
    together) plus the rows in `live_extra` (the whole published runs main() makes: Hopf N = 128
    nnGParareal, FHN-PDE d_x = 16 nnGParareal on the published paged schedule).  The rest -- minutes
    each -- are read from the newest committed profiles/rNN/published_k/*.json, written on this
    hardware by tools/published_k_run.py (the same code the -m gpu tests run,
    tests/test_gpu_published_k.py).  Every row carries its source ('live' or the file), and the
    exact-match counts are split the same way (exact_live, exact_recorded)."""
    import glob
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    import published_k as P
    rows = {}
    for name in ('burgers59_128_para', 'fhn10_512_para'):
        s, kw, pk = P.build(g, name)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = s.run(**kw)
        torch.cuda.synchronize()
        rows[name] = {'K': int(r['k']), 'published_K': pk, 'match': int(r['k']) == pk,
                      'wall_s': time.perf_counter() - t0, 'source': 'live', 'schedule': 'unpaged'}
    for name, v in (live_extra or {}).items():
        rows[name] = dict(v, source='live')
    # every round's recorded rows, the newest round's file winning per name; runs stopped at a
    # session deadline (<name>.partial.json, tools/published_k_run.py) are listed apart, not counted
    dirs = sorted(glob.glob(os.path.join(ROOT, 'profiles', 'r[0-9]*', 'published_k')))
    partial = {}
    for dr in reversed(dirs):
        for f in sorted(glob.glob(os.path.join(dr, '*.json'))):
            name = os.path.basename(f)[:-5]
            if '@' in name:   # name@seed: the seed-spread runs
                continue
            with open(f) as fh:
                d = json.load(fh)
            if name.endswith('.partial'):
                partial.setdefault(name[:-8], {'K_so_far': d['K'], 'converged': d['converged'],
                                              'published_K': d['published_K'], 'wall_s': d['wall_s'],
                                              'source': os.path.relpath(f, ROOT)})
                continue
            if name in rows:
                continue
            rows[name] = {'K': d['K'], 'published_K': d['published_K'], 'match': d['K'] == d['published_K'],
                          'wall_s': d['wall_s'], 'source': os.path.relpath(f, ROOT),
                          'schedule': 'paged' if name.endswith('_paged') else 'unpaged'}
    det = [n for n in rows if n.split('_')[2] == 'para']
    live = [n for n in rows if rows[n]['source'] == 'live']
    rec = [n for n in rows if rows[n]['source'] != 'live']
    cnt = lambda names: f"{sum(rows[n]['match'] for n in names)}/{len(names)}"
    return {'rows': rows, 'partial_runs': partial, 'parareal_exact': cnt(det), 'exact_live': cnt(live),
            'exact_recorded': cnt(rec), 'exact_all': cnt(list(rows)),
            'note': 'name = <system>_<N>_<model>[_paged]; unpaged = Nf/N RK steps per slice; paged = the '
                    'published scripts\' RK_thresh schedule (every one of 25 / 200 pages re-uses all Nf/N '
                    'steps: a 25x / 200x finer fine step). FHN-PDE d_x = 10 / 12 get 26 pages (float page '
                    'arithmetic), so their paged F integrates 4 % past every slice end and differs from the '
                    'unpaged F by 1e4 epsilon; where the pages cover the slice (d_x = 16) the two differ by '
                    '1e-13 (profiles/r06/paging_delta.txt). nnGParareal K moves with the schedule (FHN-PDE '
                    'd_x = 10: 11 paged, 9 unpaged; d_x = 12: 10 / 8), so '
                    'each row states its schedule; nnGP mismatches are discussed in DESIGN.md 5'}


def published_live(torch, g, name, reference_wall_s=None, reference_cores=None):
    """One row of the reference's published table run live, whole, at its published configuration
    (tests/published_k.py builds it from the script, file:line cited there): K against the
    published K, wall clock against the published run's where it is known."""
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    import published_k as P
    s, kw, pk = P.build(g, name)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = s.run(**kw)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    sm = P.summarise(r)
    out = {'K': sm['K'], 'published_K': pk, 'match': sm['K'] == pk, 'wall_s': wall, 'converged': sm['converged'],
           'conv_int_tail': sm['conv_int'][-6:], 'err_max': sm['err_max'], 'F_time_s': sm['F_time_s'],
           'mdl_time_s': sm['mdl_time_s'], 'schedule': 'paged' if name.endswith('_paged') else 'unpaged',
           'steps_per_slice_per_iteration': int(s.Nf / s.N) * (int(round(s.Nf / s.N / s.RK_thresh))
                                                                if s.RK_thresh != float('inf') else 1)}
    if reference_wall_s:
        out.update({'reference_wall_s': reference_wall_s, 'reference_cores': reference_cores,
                    'speedup_vs_reference_wall': reference_wall_s / wall})
    log('published live', name, json.dumps({k: out[k] for k in ('K', 'published_K', 'wall_s')}))
    return out


def hopf_fixture_check(r):
    """bench.py's Hopf solve against its oracle-loop fixture (tests/golden/hopf128_13m_nngp.npz,
    tests/golden/gen_oracle_loops.py): K, conv_int and the SHA-256 of every iterate, and the final
    state's error against the serial fine solution."""
    import hashlib
    path = os.path.join(ROOT, 'tests', 'golden', 'hopf128_13m_nngp.npz')
    if not os.path.exists(path):
        return {'fixture': None}
    P = np.load(path)
    a = np.ascontiguousarray(np.nan_to_num(np.asarray(r['u'], dtype=np.float64), nan=7.0))
    dig = hashlib.sha256(a.tobytes()).hexdigest()
    err = float(np.max(np.abs(r['u'][:, :, -1] - P['fine'])))
    return {'fixture': os.path.relpath(path, ROOT), 'K_oracle_loop': int(P['k']),
            'bitwise_oracle_loop': bool(dig == str(P['digest']) and r['k'] == int(P['k'])
                                        and list(r['conv_int']) == [int(c) for c in P['conv_int']]),
            'final_state_error_vs_serial_fine': err}


def corrections_fhn_d200(torch, g, n_pred=20):
    """nnGP corrections at the FHN-PDE d=200 shape (m=20, R=1: 1 800 fits per prediction) on a
    synthetic 3 000-row training set, one prediction after another on one GPU.  BASELINE.md §B
    derives 1.54 corrections/s for the reference's FHN d=200 N=512 run on 517 cores."""
    d, rows, m = 200, 3000, 20
    rng = np.random.default_rng(0)
    X = np.cumsum(0.02 * rng.standard_normal((rows, d)), axis=0)
    Y = 0.01 * np.sin(3 * X)
    dev = lambda a: torch.tensor(a, dtype=torch.float64, device='cuda')
    Xt, Yt = dev(X), dev(Y)
    mdl = g.NNGP_p(n=d, N=n_pred, nn=m, n_restarts=1, seed=45)
    th0 = dev(mdl.draw_thetas(n_pred + 1))
    nf = mdl.n_fits
    out = torch.empty(d, dtype=torch.float64, device='cuda')
    mdl.predict_device(Xt, Yt, rows, Xt[0] + 1e-3, th0[:nf], out=out, bias=out)   # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for j in range(n_pred):
        mdl.predict_device(Xt, Yt, rows, Xt[(37 * j) % rows] + 1e-3, th0[(j + 1) * nf:(j + 2) * nf])
    torch.cuda.synchronize()
    s = time.perf_counter() - t0
    return {'corrections_per_s': n_pred / s, 'ms_per_correction': s / n_pred * 1e3, 'd': d, 'm': m,
            'rows': rows, 'fits_per_correction': nf, 'reference_corrections_per_s_517_cores': 1.54,
            'ratio_vs_reference': n_pred / s / 1.54}


def fhn_pde_converge(torch, g, dx=20, ng=50, nf=195325):
    """BASELINE configs[4] end to end on one GPU: FHN-PDE d = 2*20^2 = 800, N = 512, nnGParareal
    m = 20 (FHN_PDE.py:175), T = 1100 (configs.py:128-139's default branch), F = RK8 with
    FHN_PDE.py's 1e8 schedule (Nf = ceil(1e8/12800)*12800 -> 195 325 steps per slice, unpaged).
    G = RK4 with 50 steps per slice: the default branch's 25 diverge at d_x = 20 (h*lambda_min =
    -3.96 for the stiffest diffusion mode, outside RK4's real stability interval [-2.79, 0]; the
    reference's own NaN guard raises 'NaN values in initial coarse solve'), and its smoke F of 25
    RK8 steps per slice diverges too."""
    ode = g.FHN_PDE(d_x=dx)
    solver = g.SolverRK(ode.get_vector_field(), Ng=ng, Nf=nf, F='RK8', G='RK4', thresh=float('inf'))
    p = g.Parareal(ode, solver, [0, 1100], 512, epsilon=5e-7, verbose=None)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = p.run(model='nngp', nn=20, seed=45)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    tm = r['timings']
    return {'wall_s': wall, 'K': r['k'], 'converged': r['converged'], 'conv_int': list(r['conv_int']),
            'F_time_s': tm['F_time'], 'G_time_s': tm['G_time'], 'mdl_time_s': tm['mdl_tot_t'],
            'd': ode.d, 'N': 512, 'Ng_per_slice': ng, 'Nf_per_slice': nf, 'm': 20,
            'spec_hits': tm.get('spec_hits', [])}


def _maxm(m):
    for M in (8, 16, 18, 20, 24, 32, 48, 64):
        if m <= M:
            return M
    return m


def _corr_inputs(d, m, rows=3000):
    """Synthetic training set and query of one correction at shape (d, m): a random walk clipped to
    the normalised box, a smooth field of it plus noise (the same inputs on the GPU and CPU legs)."""
    rng = np.random.default_rng(d + m)
    X = np.clip(np.cumsum(0.01 * rng.standard_normal((rows, d)), axis=0), -1, 1)
    Y = 0.02 * np.sin(2 * X) + 1e-5 * rng.standard_normal((rows, d))
    return X, Y, X[rows // 3] + 1e-3


def correction_roofline(torch, g, d, m, R=1, rows=3000, reps=3):
    """Roofline of one nnGP correction (NNGP_p.predict = kNN + d*9*R Nelder-Mead fits + arg-min +
    posterior mean, models.py:171-226): algorithmic flops = sum over fits of nfev x (m^3/3 + 2m^2
    + 4m) -- the jittered Cholesky, both triangular solves and the -LML sums of one likelihood
    evaluation, plus m(m+1)/2 exps counted separately -- over the correction's
    device time (HIP events on the launch stream), against the FP64 VALU peak.  The kernels run
    padded to the next instantiated size M; the executed flops at M are reported beside."""
    X, Y, qh = _corr_inputs(d, m, rows)
    dev = lambda a: torch.tensor(a, dtype=torch.float64, device='cuda')
    Xt, Yt = dev(X), dev(Y)
    mdl = g.NNGP_p(n=d, N=4, nn=m, n_restarts=R, seed=45)
    th0 = dev(mdl.draw_thetas(1))
    q = dev(qh)
    fits = torch.empty((mdl.n_fits, 4), dtype=torch.float64, device='cuda')
    preds = mdl.predict_device(Xt, Yt, rows, q, th0, fits_out=fits).clone()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        mdl.predict_device(Xt, Yt, rows, q, th0, fits_out=fits)
    b.record()
    torch.cuda.synchronize()
    sec = a.elapsed_time(b) / 1e3 / reps
    nfev = fits[:, 3].cpu().numpy()
    M = _maxm(m)
    per = m ** 3 / 3 + 2 * m ** 2 + 4 * m
    per_M = M ** 3 / 3 + 2 * M ** 2 + 4 * M
    ev = float(nfev.sum())
    tf = ev * per / sec / 1e12
    return {'d': d, 'm': m, 'R': R, 'rows': rows, 'fits': mdl.n_fits, 'ms_per_correction': sec * 1e3,
            'corrections_per_s': 1 / sec, 'fits_per_s': mdl.n_fits / sec, 'evaluations_per_s': ev / sec,
            'evaluations': ev, 'nfev_mean': float(nfev.mean()), 'nfev_max': int(nfev.max()),
            'flops_per_evaluation': per, 'exps_per_evaluation': m * (m + 1) / 2, 'padded_to': M,
            'achieved_tflops': tf, 'frac_fp64_peak': tf / FP64_PEAK_TFLOPS,
            'executed_tflops_padded': ev * per_M / sec / 1e12,
            '_preds': preds.cpu().numpy(),
            'note': 'latency-bound: a correction waits for its slowest fit (nfev_max evaluations in sequence)'}


def cpu_corrections(gpu_rows, threads):
    """BASELINE.md E.2's CPU side of the correction metric: the same corrections as
    nngp_correction_roofline (same training set, query and theta0 draws) on the host through the
    oracle's C restatement (oracle/nngp_oracle.c orc_predict: kNN + the d*9*R Nelder-Mead fits,
    OpenMP over the fits, + arg-min + posterior mean) -- corrections/s and NM fits/s beside the
    GPU's, and whether the predictions are bitwise the GPU's."""
    O = _oracle()
    out = {}
    for key, gr in gpu_rows.items():
        d, m, R, rows = gr['d'], gr['m'], gr['R'], gr['rows']
        X, Y, q = _corr_inputs(d, m, rows)
        nf = d * 9 * R
        th0 = np.random.default_rng(45).integers(-8, 0, (nf, 2)).astype(np.float64)   # NNGP_p.draw_thetas(1)
        t0 = time.perf_counter()
        reps = 0
        while True:
            preds = O.predict(X, Y, q, m, th0, n_restarts=R, nthreads=threads)
            reps += 1
            el = time.perf_counter() - t0
            if el > 1.0 or reps >= 20:
                break
        sec = el / reps
        out[key] = {'d': d, 'm': m, 'R': R, 'fits': nf, 'cpu_ms_per_correction': sec * 1e3,
                    'cpu_corrections_per_s': 1 / sec, 'cpu_fits_per_s': nf / sec,
                    'gpu_corrections_per_s': gr['corrections_per_s'], 'gpu_fits_per_s': gr['fits_per_s'],
                    'gpu_over_cpu': sec / (gr['ms_per_correction'] / 1e3),
                    'preds_bitwise_gpu': bool(np.array_equal(preds, gr['_preds'])), 'reps': reps}
    return {'rows': out, 'cpu_threads': threads, 'host_cpus_total': os.cpu_count(), 'cpu_model': cpu_model(),
            'note': 'CPU = oracle C restatement (gcc -O3 -march=x86-64-v4), OpenMP over the fits on the '
                    'threads of this process\'s CPU affinity; the reference fanned the same fits over its MPI '
                    'pool (models.py:197-202)'}


def gparareal_lorenz(torch, g):
    """Full-data GParareal (model='gpjax') on BASELINE configs[0], Lorenz N=32.  The reference's
    own run of this config (tests/golden/gp_lorenz.npz, gen_golden.py part_gp) took 247 s with
    K = 19 on the 8-core development container; that number is quoted, not re-measured here."""
    ode = g.Lorenz(normalization='-11')
    s = g.SolverRK(ode.get_vector_field(), Ng=6, Nf=450, F='RK4', G='RK4')
    p = g.Parareal(ode, s, [0, 18], 32, epsilon=5e-7, verbose=None)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = p.run(model='gpjax')
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    return {'wall_s': wall, 'K': r['k'], 'converged': r['converged'], 'mdl_time_s': r['timings']['mdl_tot_t'],
            'rows': int(r['x'].shape[0]), 'reference_K': 19, 'shim_context_wall_s_8cores': 247.0,
            'shim_context_ratio': 247.0 / wall,
            'note': 'context only, not a baseline: the 247 s is the reference run under this repo\'s numpy '
                    'stand-in for jax (tests/golden/jaxshim) on the 8-core development container, '
                    'not the reference\'s own jax/XLA path'}


def gparareal_burgers(torch, g):
    """Full-data GParareal (model='gpjax', models.py:273-473) at BASELINE scale: Burgers d=128
    N=128 T=5 on Burgers_perf_across_m.py's 2 000-step schedule.  Training rows grow to ~750; every
    Nelder-Mead round factors one (rows+1)^2 matrix per unfinished fit of the d*9 = 1 152 (batched
    blocked Cholesky, nngp_gpfull.hip).  The published GParareal run (Burges_scal_final_5_128_gp,
    Burgers.py's paged schedule) converged in K = 6.  FP64 rate: the training's Cholesky flops,
    sum over rounds of (active fits) x (rows+1)^3/3, are bounded above by 400 rounds x 1 152 fits
    per call; the upper bound over the training time is reported against the FP64 peak, and beside
    it the executed rate: each fit's nfev counts the matrices it factored, so the training's
    Cholesky flops are sum over calls of (sum of nfev) x (rows+1)^3/3 (n^3/3, the dominant term)."""
    ode = g.Burgers(d_x=128, normalization='-11')
    s = g.SolverRK(ode.get_vector_field(), Ng=4, Nf=2000, F='RK8', G='RK1')
    p = g.Parareal(ode, s, [0, 5], 128, epsilon=5e-7, verbose=None)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = p.run(model='gpjax', add_model=True)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    mdl = r['mdl']
    rows, K = [], r['k']
    n_rows, I = 0, 0
    for k in range(K):   # training rows at iteration k: sum over iterations of N - I_k + 1
        n_rows += 128 - I + 1 - 1
        rows.append(n_rows)
        I = r['conv_int'][k] if k < len(r['conv_int']) else I
    train = [float(v) for v in mdl.tot_train_t[:K]]
    ub = sum(rd * 1152 * (n + 1) ** 3 / 3 for rd, n in zip(mdl.rounds, rows))
    # executed: every likelihood evaluation factors one (rows+1)^2 matrix, (rows+1)^3/3 flops
    # (the sum of the fits' nfev per training call)
    ex = sum(e * (n + 1) ** 3 / 3 for e, n in zip(mdl.call_evals, mdl.call_rows))
    return {'wall_s': wall, 'K': K, 'reference_K': 6, 'converged': r['converged'], 'conv_int': list(r['conv_int']),
            'F_time_s': r['timings']['F_time'], 'mdl_time_s': r['timings']['mdl_tot_t'],
            'training_rows_per_iteration': rows, 'nm_rounds_per_iteration': list(mdl.rounds),
            'training_s_per_iteration': train,
            'cholesky_tflops_upper_bound': ub / max(sum(train), 1e-9) / 1e12,
            'frac_fp64_peak_upper_bound': ub / max(sum(train), 1e-9) / 1e12 / FP64_PEAK_TFLOPS,
            'evaluations_per_call': list(mdl.call_evals), 'rows_per_call': list(mdl.call_rows),
            'cholesky_tflops_executed': ex / max(sum(train), 1e-9) / 1e12,
            'frac_fp64_peak_executed': ex / max(sum(train), 1e-9) / 1e12 / FP64_PEAK_TFLOPS}


def gpfull_round_roofline(torch, g, shapes=((4096, 240), (9500, 27), (753, 1152)), reps=3):
    """One batched full-GP -LML evaluation = one GParareal Nelder-Mead round (nngp_gpfull_lml:
    the left-looking 64-column Cholesky of every point's (rows+1)^2 matrix) at the
    shapes the published runs reach -- FHN-PDE d_x = 10 (240 of its 1 800 matrices per slab),
    Hopf N = 512, Burgers N = 128 -- with a jitter that lets every factor complete, so the executed
    flops are exactly points x (rows+1)^3 / 3 (bound: the FP64 matrix cores, 78.6 TF/s)."""
    import ctypes
    out = {}
    ip, dp = ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_double)
    for n, npts in shapes:
        rng = np.random.default_rng(n)
        x = rng.uniform(-1, 1, (n, 3))
        X = torch.tensor(x, device='cuda')
        Y = torch.tensor(np.sin(2 * x), device='cuda')
        c = np.ascontiguousarray(np.arange(npts) % 3, dtype=np.int32)
        jx = np.full(npts, -2.0)
        th = np.ascontiguousarray(np.column_stack([0.3 + 0.5 * rng.random(npts), 0.5 + rng.random(npts)]))
        fv = np.empty(npts)
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g._lib.check(g.lib().nngp_gpfull_lml(X.data_ptr(), n, 3, Y.data_ptr(), npts, c.ctypes.data_as(ip),
                                                 jx.ctypes.data_as(dp), th.ctypes.data_as(dp), fv.ctypes.data_as(dp),
                                                 None, None))
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        t = min(ts)
        fl = npts * (n + 1) ** 3 / 3
        out[f'{n}x{npts}'] = {'ms': t * 1e3, 'tflops': fl / t / 1e12, 'frac_fp64_peak': fl / t / 1e12 / FP64_PEAK_TFLOPS,
                              'all_finite': bool(np.isfinite(fv).all())}
    log('gpfull round roofline', json.dumps(out))
    return out


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import oracle as O
    return O


def cpu_threads():
    return int(os.environ.get('OMP_NUM_THREADS', '0') or 0) or len(os.sched_getaffinity(0))


def cpu_model():
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_single_core(budget_s=0.4):
    """One host core's us per fine step of the CPU restatement (oracle/nngp_oracle.c, gcc -O3
    -march=x86-64-v4), next to the reference's per-core figures (its XLA-CPU path,
    one MPI worker core per slice).  PDE fields twice: the stencil port and the reference's dense
    formulation (Dxx@u / (a L)@u1 as full matrices, systems.py:321-446 -- the same results, bit
    for bit, at the reference's d^2 cost).  The BASELINE.md E sanity bar: within ~2x."""
    O = _oracle()
    x128 = np.linspace(-1, 1, 128)
    rng = np.random.default_rng(0)
    cases = [
        ('hopf_rk8', lambda dn: O.System('hopf', param=(500.0,)), 8, np.array([0.1, 0.1, -0.9]), 0.80),
        ('tomlab_rk4', lambda dn: O.System('tomlab'), 4, np.array([0.3, 0.1, -0.2]), 0.30),
        ('burgers_d128_rk8', lambda dn: O.System('burgers', d=128, param=(0.01,), mn=0.0, mx=1.0, dense=dn), 8,
         0.5 * (np.cos(4.5 * np.pi * x128) + 1) * 2 - 1, 46.6),
        ('fhn_pde_d200_rk8', lambda dn: O.System('fhn_pde', nx=10, mn=-1, mx=1, dense=dn), 8,
         rng.uniform(-0.5, 0.5, 200), 39.9),
        ('fhn_pde_d512_rk8', lambda dn: O.System('fhn_pde', nx=16, mn=-1, mx=1, dense=dn), 8,
         rng.uniform(-0.5, 0.5, 512), 425.0),
    ]
    res = {}
    for name, mk, order, u0, ref in cases:
        for dense in ((False, True) if name.startswith(('burgers', 'fhn')) else (False,)):
            s = mk(dense)
            U = u0.reshape(1, -1)
            probe = 8
            t0 = time.perf_counter()
            s.rk_batch(order, [0.0], [1e-3 * probe], probe, U, nthreads=1)
            per = (time.perf_counter() - t0) / probe
            steps = int(max(probe, min(2_000_000, budget_s / max(per, 1e-9))))
            t0 = time.perf_counter()
            s.rk_batch(order, [0.0], [1e-3 * steps], steps, U, nthreads=1)
            us = (time.perf_counter() - t0) / steps * 1e6
            key = name + ('_dense' if dense else ('_stencil' if name.startswith(('burgers', 'fhn')) else ''))
            ratio = ref / us
            res[key] = {'us_per_step': us, 'steps_timed': steps, 'reference_us_per_step': ref,
                        'reference_over_port': ratio, 'within_2x_band': bool(0.5 <= ratio <= 2.0)}
    res['note'] = ('BASELINE.md E.2 asks the CPU port to land within ~2x of the reference\'s per-core '
                   'figures; entries with within_2x_band false are outside it -- the port is faster per '
                   'core than the published XLA-CPU path (gcc -O3 AVX-512 C against jitted Python), so '
                   'GPU/CPU ratios built on it understate the speed-up over the reference itself')
    return res


def cpu_baseline(steps_per_slice_full, n_slices, target_s=10.0):
    """Oracle C restatement (OpenMP over slices) on a bounded sample of the fine sweep."""
    O = _oracle()
    threads = cpu_threads()
    s = O.System('hopf', param=(500.0,))
    rng = np.random.default_rng(1234)
    U = rng.uniform(-0.5, 0.5, size=(n_slices, 3))
    t = np.linspace(-20, 500, n_slices + 1)
    probe = 20000
    t0 = time.perf_counter()
    s.rk_batch(4, t[:-1], t[1:], probe, U, nthreads=threads)
    dt = time.perf_counter() - t0
    steps = int(min(steps_per_slice_full, max(probe, probe * target_s / max(dt, 1e-6))))
    t0 = time.perf_counter()
    s.rk_batch(4, t[:-1], t[1:], steps, U, nthreads=threads)
    dt = time.perf_counter() - t0
    return {'value': n_slices * steps / dt, 'unit': 'fine RK steps/s', 'cores': threads, 'kind': 'port',
            'sample': f'{n_slices} Hopf slices x {steps} RK4 steps (of {steps_per_slice_full}), '
                      f'{dt:.1f} s, oracle/nngp_oracle.c gcc -O3 -march=x86-64-v4 OpenMP',
            'cpu_model': cpu_model(), 'host_cpus_total': os.cpu_count(),
            'cores_note': f'{threads} threads = the CPU affinity this process was given '
                          f'(len(sched_getaffinity)), not the {os.cpu_count()} CPUs the machine reports'}


def burgers_cpu_converge(threads):
    """CPU baseline for the north star's Burgers target, measured to convergence: the oracle's C
    restatement runs the whole nnGParareal solve of the same config (OpenMP over slices for F and
    over the 1 152 fits of each correction), F in the reference's dense formulation (Dxx@u,
    Dx@u as 128 x 128 matrices, systems.py:421-446; bit-identical to the stencil).  Returns
    (wall s, F s, result)."""
    O = _oracle()
    s = O.System('burgers', d=128, param=(0.01,), mn=0.0, mx=1.0, dense=True)
    x = np.linspace(-1, 1, 128)
    u0 = s.fit(0.5 * (np.cos(4.5 * np.pi * x) + 1))
    f_time = [0.0]
    rk_batch = s.rk_batch

    def timed(*a, **k):
        t = time.perf_counter()
        out = rk_batch(*a, **k)
        f_time[0] += time.perf_counter() - t
        return out
    s.rk_batch = timed
    t0 = time.perf_counter()
    r = O.parareal(s, [0, 5], 128, 4, 2000, 'RK1', 'RK8', model='nngp', nn=15, seed=45, u0=u0, nthreads=threads)
    return time.perf_counter() - t0, f_time[0], r


def burgers_published_schedule(torch, g, sample_pages=2):
    """The published Burgers N=128 scalability run (Burgers.py:29-33, 95-108: Nf = N*4*10^4 total
    RK8 steps, RK_thresh = Nf/N/200) pages every slice into 200 pages that each re-use the full
    39 999-step count (new_lib.py:57-69): 7 999 800 RK8 steps per slice per
    iteration.  Time `sample_pages` of those pages for all 128 slices (LINSPACE grids, as the
    legacy RK_last integrates) and scale to the iteration; the reference's own F time per
    iteration on 128 worker cores was 372.8 s."""
    ode = g.Burgers(d_x=128, normalization='-11')
    solver = g.SolverRK(ode.get_vector_field(), Ng=4, Nf=39999, F='RK8', G='RK1', step_mode='linspace',
                        thresh=float('inf'))
    n, pages = 128, 200
    t = np.linspace(0, 5, n + 1)
    step = (t[1:] - t[:-1]) / 40000
    dev = lambda a: torch.tensor(a, dtype=torch.float64, device='cuda')
    U = dev(np.tile(ode.get_init_cond(), (n, 1)))
    out = torch.empty_like(U)
    solver.run_F_batch(dev(t[:-1]), dev(t[:-1] + step * 200), U, out=out)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    ts = t[:-1].copy()
    for _ in range(sample_pages):
        te = ts + step * 200
        solver.run_F_batch(dev(ts), dev(te), U, out=out)
        U, out = out, U
        ts = te
    b.record()
    torch.cuda.synchronize()
    per_page = a.elapsed_time(b) / 1e3 / sample_pages
    it = per_page * pages
    return {'F_per_iteration_s': it, 'reference_F_per_iteration_s': 372.8, 'speedup_vs_reference_F': 372.8 / it,
            'steps_per_slice': pages * 39999, 'sample': f'{sample_pages} of {pages} pages x 128 slices, RK8, linspace',
            'us_per_step': per_page / 39999 * 1e6}


def ode_published_schedule(torch, g, ode, n, tspan, tab, eff, ref_s, ref_cores, sample_steps, fma=False):
    """One ODE's published scalability schedule: time `sample_steps` of its `eff` effective fine
    steps per slice per iteration for all n slices (LINSPACE grids as the legacy RK_last, lane-group
    kernel) and scale to the iteration, next to the reference's F time per iteration on its
    cluster.  Each slice is one serial chain, so this compares per-step latency: a
    CPU core per slice there, one GPU lane group per slice here.  fma=True: the opt-in contracted
    propagator (SolverRK(fma=True), tests/test_gpu_contract.py's 1e-12 tolerance)."""
    d = len(ode.get_init_cond())
    solver = g.SolverRK(ode.get_vector_field(), Ng=10, Nf=sample_steps, F=tab, G='RK1',
                        step_mode='linspace', thresh=float('inf'), fma=fma)
    small = g.SolverRK(ode.get_vector_field(), Ng=10, Nf=1000, F=tab, G='RK1', step_mode='linspace',
                       thresh=float('inf'), fma=fma)
    t = np.linspace(tspan[0], tspan[1], n + 1)
    dev = lambda a: torch.tensor(a, dtype=torch.float64, device='cuda')
    rng = np.random.default_rng(0)
    U = dev(rng.uniform(-0.5, 0.5, (n, d)))
    out = torch.empty_like(U)
    small.run_F_batch(dev(t[:-1]), dev(t[1:]), U, out=out)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    solver.run_F_batch(dev(t[:-1]), dev(t[1:]), U, out=out)
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1e3 / sample_steps
    it = us * 1e-6 * eff
    return {'us_per_step': us, 'F_per_iteration_s': it, 'reference_F_per_iteration_s': ref_s,
            'reference_cores': ref_cores, 'speedup_vs_reference_F': ref_s / it, 'steps_per_slice': eff,
            'sample': f'{sample_steps} of {eff:.3g} steps x {n} slices, {tab}, linspace',
            'build': 'contracted (opt-in, 1e-12)' if fma else 'exact (bitwise the oracle)'}


def tomlab_published_schedule(torch, g, sample_steps=1_000_000, fma=False):
    """Thomas labyrinth N=256 (TomLab.py:83-101: Nf = Ng*ceil(1e9/Ng), RK4, RK_thresh = Nf/N/109):
    110 pages of the full per-slice count (new_lib.py:57-69) = 4.30e8 RK4 steps per
    slice per iteration; the reference's F per iteration on 282 cores was 156 s, 0.30-0.37 us/step."""
    return ode_published_schedule(torch, g, g.ThomasLabyrinth(normalization='-11'), 256, (0, 100), 'RK4',
                                  4.30e8, 156.0, 282, sample_steps, fma)


def hopf_published_schedule(torch, g, sample_steps=500_000, fma=False):
    """Hopf N=128 (Hopf.py:60-69: Nf x 10^4, RK8, RK_thresh = Nf/N/25): 3.4e8 effective RK8 steps per
    slice per iteration (272 s / 0.80 us); the reference's F per iteration on 141
    cores was 272 s."""
    return ode_published_schedule(torch, g, g.Hopf(normalization='-11'), 128, (-20, 500), 'RK8',
                                  3.4e8, 272.0, 141, sample_steps, fma)


def fhn_pde_fine_sweeps(torch, g):
    """FHN-PDE N=512 fine sweeps on the field kernel (RK8, all 512 slices in one launch):
    - d=200 (d_x=10) on the published schedule (FHN_PDE.py:146-161, legacy linspace grids, '-11'
      with +-1 bounds): 5.08e6 effective RK8 steps per slice per iteration; the
      reference's F per iteration on 517 cores was 202 s;
    - d=800 (d_x=20), BASELINE configs[4]: 195 325 RK8 steps per slice per iteration (SURVEY.md
      §8d), with the achieved FP64 rate against the VALU peak (215 600 flops per step per slice).
    A sample of steps is timed for all 512 slices and scaled to the iteration."""
    dev = lambda a: torch.tensor(a, dtype=torch.float64, device='cuda')
    res = {}
    for nx, mode, norm, sample, eff, ref in ((10, 'linspace', '-11', 10000, 5.08e6, 202.0),
                                             (20, 'fixed', None, 2000, 195325, None)):
        ode = g.FHN_PDE(d_x=nx, normalization=norm) if norm else g.FHN_PDE(d_x=nx)
        n, d = 512, 2 * nx * nx
        solver = g.SolverRK(ode.get_vector_field(), Ng=1, Nf=sample, F='RK8', G='RK1', step_mode=mode,
                            thresh=float('inf'))
        t = np.linspace(0, 1100, n + 1)
        rng = np.random.default_rng(0)
        U = dev(np.clip(ode.get_init_cond()[None, :] + 0.01 * rng.standard_normal((n, d)), -1, 1))
        out = torch.empty_like(U)
        solver.run_F_batch(dev(t[:-1]), dev(t[1:]), U, out=out)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        solver.run_F_batch(dev(t[:-1]), dev(t[1:]), U, out=out)
        b.record()
        torch.cuda.synchronize()
        sec = a.elapsed_time(b) / 1e3
        us = sec / sample * 1e6
        flops = 15.5 * d * 11 + (2 * 39 + 11 + 2 * 5) * d   # S*F_rhs + (2nnz(a)+S+2nnz(b))*d
        tf = n * sample * flops / sec / 1e12
        r = {'d': d, 'slices': n, 'us_per_step': us, 'steps_per_s': n * sample / sec, 'tflops': tf,
             'frac_fp64_peak': tf / FP64_PEAK_TFLOPS, 'steps_per_slice_per_iteration': eff,
             'F_per_iteration_s': us * 1e-6 * eff, 'sample': f'{sample} RK8 steps x 512 slices, {mode}'}
        if ref:
            r.update({'reference_F_per_iteration_s': ref, 'reference_cores': 517,
                      'speedup_vs_reference_F': ref / (us * 1e-6 * eff)})
        res[f'd{d}'] = r
    return res


def fhn_strong(torch, g, world, rank, steps=3, warmup=1, sample=400, n_pred=4):
    """The north star's strong-scaling workload, FHN-PDE d=800 (d_x=20), N=512 slices, at every
    world size: the fine sweep of all 512 slices sharded into contiguous blocks (512/world per
    rank, fine_sweep_sharded) + the all-gather of the end states, and the nnGP correction of one
    slice with its 7 200 fits sharded by coordinate (nngp_predict_range, 800/world coordinates
    per rank) + the all-gather of the predictions.  Timed between barriers, max over ranks.
    Projected iteration = F (195 325 RK8 steps per slice, FHN_PDE.py's 1e8 schedule) + 511
    corrections.  At world = 1 the 8-GPU per-rank shares are also measured on this GPU (64
    slices; 100 of the 800 coordinates), giving the projected 1 -> 8 speed-up."""
    import ctypes
    from nngp_amd.models import JITTERS
    from nngp_amd.parareal import shard_bounds
    dist = torch.distributed
    n_sl, nx = 512, 20
    d = 2 * nx * nx
    steps_it = 195325
    ode = g.FHN_PDE(d_x=nx)
    solver = g.SolverRK(ode.get_vector_field(), Ng=50, Nf=sample, F='RK8', G='RK4', thresh=float('inf'))
    dev = lambda a: torch.tensor(a, dtype=torch.float64, device='cuda')
    rng = np.random.default_rng(0)
    t = np.linspace(0, 1100, n_sl + 1)
    U = np.clip(ode.get_init_cond()[None, :] + 0.01 * rng.standard_normal((n_sl, d)), -1, 1)
    Ud, td = dev(U), dev(t)
    UF = torch.empty((n_sl + 1, d), dtype=torch.float64, device='cuda')
    Ufull = torch.empty((n_sl + 1, d), dtype=torch.float64, device='cuda')
    Ufull[:n_sl] = Ud
    group = None if world > 1 else None
    prop = lambda a, b, u, out: solver.run_F_batch(a, b, u, out=out)

    def sweep():
        if world > 1:
            g.parareal.fine_sweep_sharded(prop, td, Ufull, UF, 0, n_sl, group)
        else:
            solver.run_F_batch(td[:-1], td[1:], Ud, out=UF[1:])

    def timed(fn, k):
        barrier_sync(torch, world)
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        barrier_sync(torch, world)
        el = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([el], dtype=torch.float64, device='cuda')
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = float(tt.item())
        return el / k

    for _ in range(warmup):
        sweep()
    f_s = timed(sweep, steps)
    # nnGP correction of one slice, coordinate-sharded over the ranks (same data on every rank)
    rows, m = 3000, 20
    X = np.clip(np.cumsum(0.01 * rng.standard_normal((rows, d)), axis=0), -1, 1)
    Y = 0.02 * np.sin(2 * X)
    mdl = g.NNGP_p(n=d, N=4, nn=m, n_restarts=1, seed=45)
    th0 = dev(mdl.draw_thetas(1))
    Xd, Yd = dev(X), dev(Y)
    jit = np.ascontiguousarray(JITTERS)
    jp = jit.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    lib = g.lib()
    c0, c1, chunk = shard_bounds(0, d, world, rank)
    send = torch.zeros(chunk, dtype=torch.float64, device='cuda')
    qs = [Xd[(97 * j) % rows] + 1e-3 for j in range(n_pred)]
    st = torch.cuda.current_stream().cuda_stream

    def range_pred(q, a, b, out):
        g._lib.check(lib.nngp_predict_range(Xd.data_ptr(), Yd.data_ptr(), rows, d, q.data_ptr(), m, len(jit), jp, 1,
                                            th0.data_ptr(), a, b, 0.1, 0.1, 400, out.data_ptr(), st))

    def corrections():
        for q in qs:
            if c1 > c0:
                range_pred(q, c0, c1, send[:c1 - c0])
            if world > 1:
                g.parareal._all_gather_flat(send, None, world)

    corrections()
    c_s = timed(corrections, 1) / n_pred
    sweep_res = sharded_sweep_timing(torch, g, solver, td, Ufull, Xd, Yd, rows, mdl, world, rank, timed)
    res = {'workload': 'FHN-PDE d=800 (d_x=20) N=512, RK8 fine sweep + coordinate-sharded nnGP corrections (m=20)',
           'world': world, 'slices_per_rank': (n_sl + world - 1) // world,
           'F_us_per_step': f_s / sample * 1e6, 'F_steps_per_s': n_sl * sample / f_s,
           'correction_ms': c_s * 1e3, 'corrections_per_s': 1 / c_s,
           'iteration_s_projected': f_s / sample * steps_it + (n_sl - 1) * c_s,
           'sample': f'{sample} RK8 steps x 512 slices; {n_pred} corrections of 7200 fits (rows {rows})',
           'correction_sweep': sweep_res}
    if world == 1:   # the 8-GPU per-rank shares, measured on this GPU
        sh = 64
        sweep8 = lambda: solver.run_F_batch(td[:sh], td[1:sh + 1], Ud[:sh].contiguous(), out=UF[1:sh + 1])
        sweep8()
        f8 = timed(sweep8, steps)
        out8 = torch.empty(100, dtype=torch.float64, device='cuda')

        def corr8():
            for q in qs:
                range_pred(q, 0, 100, out8)
        corr8()
        c8 = timed(corr8, 1) / n_pred
        it1 = res['iteration_s_projected']
        it8 = f8 / sample * steps_it + (n_sl - 1) * c8
        res['per_rank_share_8gpu'] = {'F_us_per_step_64_slices': f8 / sample * 1e6,
                                      'correction_ms_100_coords': c8 * 1e3,
                                      'iteration_s_projected_8gpu': it8,
                                      'projected_speedup_1_to_8': it1 / it8,
                                      'projected_F_speedup_1_to_8': f_s / f8,
                                      'note': 'excludes the per-iteration all-gather (3.3 MB) and the '
                                              'per-slice all-gather of 800 predictions (6.4 KB)'}
    return res


def sharded_sweep_timing(torch, g, solver, td, Ufull, Xd, Yd, rows, mdl, world, rank, timed, n_sw=8):
    """The sequential correction sweep (parareal.py:359-382) over n_sw consecutive FHN-PDE d=800
    slices (G = RK4 50 steps, m = 20, 7 200 fits per prediction), two ways:
    - 'python_loop': the launches issued one by one from Python per slice -- G, this rank's
      coordinates (nngp_predict_range), the all-gather of the predictions (torch.distributed),
      u = preds + uG (parareal.correction_sweep_sharded's pattern);
    - 'native': ONE library call for the whole sweep -- nngp_correction_sweep_sharded over the
      library's RCCL communicator when the job has more than one rank, nngp_correction_sweep
      (speculation off) on one rank.
    The difference per slice is the host overhead the native call removes."""
    import ctypes
    from nngp_amd.models import JITTERS
    from nngp_amd.parareal import shard_bounds
    lib = g.lib()
    d = Xd.shape[1]
    m, nf = 20, mdl.n_fits
    jit = np.ascontiguousarray(JITTERS)
    jp = jit.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    th = torch.tensor(mdl.draw_thetas(n_sw), dtype=torch.float64, device='cuda')
    cs = solver.f.csystem(Xd.device)
    st = torch.cuda.current_stream().cuda_stream
    U1 = Ufull.clone()
    UG1 = torch.empty_like(U1)
    zeros = torch.zeros(d, dtype=torch.float64, device='cuda')
    c0, c1, chunk = shard_bounds(0, d, world, rank)
    gather = torch.zeros(world * chunk, dtype=torch.float64, device='cuda')
    # the library's communicator only when opted in (NNGP_NATIVE_COMM=1, as Parareal); otherwise
    # the 'native' leg is the unsharded sweep on every rank
    comm = world > 1 and g.parareal.native_comm_default() and g._lib.comm_for(None)

    send = torch.zeros(chunk, dtype=torch.float64, device='cuda')

    def python_loop():
        for i in range(n_sw):
            solver.run_G_batch(td[i:i + 1], td[i + 1:i + 2], U1[i:i + 1], out=UG1[i + 1:i + 2])
            if c1 > c0:
                g._lib.check(lib.nngp_predict_range(Xd.data_ptr(), Yd.data_ptr(), rows, d, U1[i].data_ptr(), m,
                                                    len(jit), jp, 1, th[i * nf:(i + 1) * nf].data_ptr(), c0, c1,
                                                    0.1, 0.1, 400, send.data_ptr(), st))
            if world > 1:
                torch.distributed.all_gather_into_tensor(gather, send)
            else:
                gather.copy_(send)
            g._lib.check(lib.nngp_parareal_update(d, gather.data_ptr(), zeros.data_ptr(), UG1[i + 1].data_ptr(),
                                                  U1[i + 1].data_ptr(), st))

    def native():
        if comm:
            g._lib.check(lib.nngp_correction_sweep_sharded(
                ctypes.byref(cs), 4, 0, 50, td.data_ptr(), 0, n_sw, U1.data_ptr(), UG1.data_ptr(), Xd.data_ptr(),
                Yd.data_ptr(), rows, m, len(jit), jp, 1, th.data_ptr(), 0.1, 0.1, 400, gather.data_ptr(), None, st))
        else:
            scratch = torch.empty(d, dtype=torch.float64, device='cuda')
            g._lib.check(lib.nngp_correction_sweep(
                ctypes.byref(cs), 4, 0, 50, td.data_ptr(), 0, n_sw, U1.data_ptr(), UG1.data_ptr(), None, None,
                g._lib.MODEL_NNGP, Xd.data_ptr(), Yd.data_ptr(), rows, m, len(jit), jp, 1, th.data_ptr(), 0.1, 0.1,
                400, scratch.data_ptr(), 0, None, None, st))

    out = {}
    finals = {}
    for name, fn in (('python_loop', python_loop), ('native', native)):
        fn()
        out[f'{name}_ms_per_slice'] = timed(fn, 2) / n_sw * 1e3
        torch.cuda.synchronize()
        finals[name] = U1.clone()
    out['host_overhead_ms_per_slice_removed'] = out['python_loop_ms_per_slice'] - out['native_ms_per_slice']
    # the two paths compute the same sweep from the same U1[0]: bitwise equal on every rank
    same = torch.tensor([1 if torch.equal(finals['python_loop'], finals['native']) else 0], dtype=torch.int32,
                        device='cuda')
    if world > 1:
        torch.distributed.all_reduce(same, op=torch.distributed.ReduceOp.MIN)
    out['native_bitwise_python_loop'] = bool(same.item())
    out['native_path'] = ('nngp_correction_sweep_sharded (library RCCL communicator)' if comm
                          else 'nngp_correction_sweep (unsharded, every rank)')
    out['slices'] = n_sw
    return out


def read_traffic():
    """HBM bytes per launch of the fine kernel from the NEWEST committed PMC passes
    (profiles/rNN/fine_kernel_traffic.json, written by tools/pmc_traffic.py from rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes of tools/pmc_probe.py): FETCH_SIZE x 2 (the guide's gfx950
    correction) + WRITE_SIZE, median over the headline-length launches, every launch beside it,
    and the same window's bytes under a null kernel (the device's background).  Returns
    (summary dict, source path) or (None, None)."""
    import glob
    import re
    cands = []
    for p in glob.glob(os.path.join(ROOT, 'profiles', 'r[0-9]*', 'fine_kernel_traffic.json')):
        m = re.search(r'r(\d+)', os.path.basename(os.path.dirname(p)))
        cands.append((int(m.group(1)), p))
    if not cands:
        return None, None
    path = max(cands)[1]
    try:
        t = json.load(open(path))
    except Exception:
        return None, None
    if 'bytes_per_launch_all' not in t:   # pre-round-3 format (no x2 correction, no null kernel)
        return None, None
    return {'traffic': t['bytes_per_launch'], 'traffic_all_launches': t['bytes_per_launch_all'],
            'traffic_short_launches': t.get('bytes_per_launch_short'),
            'traffic_null_kernel_same_window': t.get('null_kernel_bytes_median'),
            'traffic_correction': t.get('fetch_correction')}, os.path.relpath(path, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--steps-per-slice', type=int, default=2048 * 85 * 10000 // 128)   # 13.6e6
    ap.add_argument('--slices-per-gpu', type=int, default=128)
    ap.add_argument('--no-extras', action='store_true', help='skip corrections/convergence/CPU legs')
    ap.add_argument('--workload', choices=['hopf', 'fhn_pde'], default='hopf',
                    help="headline value: 'hopf' = BASELINE configs[1] Hopf fine sweep, weak scaling "
                         "(128 slices per GPU); 'fhn_pde' = FHN-PDE d=800 N=512 fine sweep, strong "
                         "scaling (512 slices over all GPUs; the north star's 1->8 target)")
    ap.add_argument('--dry-run', action='store_true',
                    help='launcher check without a GPU: the same N-rank launch and process group (gloo), '
                         'no kernels; prints the JSON line with value null')
    args = ap.parse_args()
    if args.gpus < 1:
        sys.exit('bench.py: --gpus must be >= 1')
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    import torch
    world, rank = dist_init(args.gpus, args.dry_run)
    if args.dry_run:
        t0 = time.perf_counter()
        if world > 1:
            torch.distributed.barrier()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
        if world > 1:
            torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
            ranks = [None] * world
            torch.distributed.all_gather_object(ranks, rank)
            torch.distributed.destroy_process_group()
        else:
            ranks = [0]
        if rank == 0:
            print(json.dumps({'metric': 'fine RK steps/sec (+ nnGP corrections/sec; wall-clock to convergence)',
                              'value': None, 'unit': 'fine RK steps/s', 'n_gpus': world, 'dry_run': True,
                              'ranks_seen': ranks, 'barrier_s_max': float(el.item())}), flush=True)
        return
    import nngp_amd as g
    g.lib()

    elapsed, kernel_s, n_total, _, gather_path, native_check = fine_sweep_bench(
        torch, g, world, rank, args.steps, args.warmup, args.steps_per_slice, args.slices_per_gpu)
    total_steps = n_total * args.steps_per_slice * args.steps
    value = total_steps / elapsed
    flops_launch = FLOPS_PER_STEP[('hopf', 'RK4')] * args.steps_per_slice * args.slices_per_gpu
    achieved_tf = flops_launch / kernel_s / 1e12
    tr, tr_src = read_traffic()
    traffic = tr['traffic'] if tr else None
    res = {
        'metric': 'fine RK steps/sec (+ nnGP corrections/sec; wall-clock to convergence)',
        'value': value, 'unit': 'fine RK steps/s', 'n_gpus': world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': elapsed / args.steps * 1e3, 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f64', 'data': 'synthetic',
        'config': {'workload': 'nonautonomous Hopf (Hopf.py), RK4 fine sweep, 13.6e6 steps/slice',
                   'slices_per_gpu': args.slices_per_gpu, 'total_slices': n_total,
                   'steps_per_slice': args.steps_per_slice, 'parallelism': f'time-slices x{world}',
                   'allgather': gather_path, 'native_allgather_check': native_check},
        'roofline': {'bound': 'fp64-valu', 'achieved': achieved_tf, 'peak': FP64_PEAK_TFLOPS,
                     'unit': 'TFLOP/s', 'frac': achieved_tf / FP64_PEAK_TFLOPS, 'traffic': traffic,
                     **({k: v for k, v in tr.items() if k != 'traffic'} if tr else {}), 'traffic_source': tr_src,
                     'hbm_GBps': (traffic / kernel_s / 1e9) if traffic else None, 'hbm_peak_GBps': HBM_PEAK_GBS,
                     'algorithmic_bytes_per_launch': args.slices_per_gpu * (2 * 3 * 8 + 2 * 8),
                     'kernel': 'rk_group_kernel<HOPF,RK4>', 'kernel_ms': kernel_s * 1e3,
                     'issue_floor_us_per_step': LANE_VALU_PER_STEP * CYCLES_PER_F64_VALU / (SHADER_GHZ * 1e3),
                     'us_per_step': kernel_s / args.steps_per_slice * 1e6,
                     'issue_floor_frac': (LANE_VALU_PER_STEP * CYCLES_PER_F64_VALU / (SHADER_GHZ * 1e9))
                                         / (kernel_s / args.steps_per_slice),
                     'flops_per_step_per_slice': FLOPS_PER_STEP[('hopf', 'RK4')]},
    }
    # the strong-scaling workload (FHN-PDE N=512), measured at every world size
    strong = fhn_strong(torch, g, world, rank)
    res['fhn_pde_strong'] = strong
    if args.workload == 'fhn_pde':
        res.update({'value': strong['F_steps_per_s'], 'scaling': 'strong',
                    'ms_per_step': strong['F_us_per_step'] * 400 / 1e3,
                    'config': {'workload': strong['workload'], 'total_slices': 512, 'd': 800,
                               'slices_per_gpu': strong['slices_per_rank'], 'parallelism': f'time-slices x{world}'}})
    if rank == 0 and world == 1 and not args.no_extras:
        n_pred, pred_s, _ = corrections_bench(torch, g)
        res['nngp_corrections_per_s'] = n_pred / pred_s
        res['nngp_correction_ms'] = pred_s / n_pred * 1e3
        runs = {}
        for which in ('burgers', 'hopf'):
            wall, k, conv, tim, runs[which] = converge(torch, g, which)
            res[f'{which}_n128_to_convergence'] = {'wall_s': wall, 'K': k, 'converged': conv,
                                                   'F_time_s': tim['F_time'], 'mdl_time_s': tim['mdl_tot_t'],
                                                   'conv_int': tim.get('conv_int', []),
                                                   'spec_hits': tim.get('spec_hits', [])}
            log(which, 'converged', conv, 'K', k, f'{wall:.2f}s')
        res['hopf_n128_to_convergence'].update(hopf_fixture_check(runs['hopf']))
        res['nngp_corrections_fhn_d200'] = corrections_fhn_d200(torch, g)
        res['nngp_correction_roofline'] = {f'd{d}_m{m}_R{R}': correction_roofline(torch, g, d, m, R)
                                           for d, m, R in ((800, 20, 1), (200, 20, 1), (128, 15, 1), (3, 15, 2))}
        log('correction roofline', json.dumps({k: {a: b for a, b in v.items() if a != '_preds'}
                                                for k, v in res['nngp_correction_roofline'].items()}))
        res['nngp_corrections_hopf_vs_reference'] = {'reference_corrections_per_s_141_cores': 44.0,
                                                      'ratio': res['nngp_corrections_per_s'] / 44.0}
        res['fhn_pde_n512_to_convergence'] = fhn_pde_converge(torch, g)
        log('fhn-pde d=800 N=512', json.dumps(res['fhn_pde_n512_to_convergence']))
        # two whole published runs, live: Hopf N = 128 nnGParareal (Hopf.py, K = 13 in 3 565 s on 141
        # cores) and FHN-PDE d_x = 16 nnGParareal on the published PAGED schedule (FHN_PDE.py:146-175:
        # 25 pages x 195 324 RK8 steps per slice per iteration, K = 6 in 17 849 s on 517 cores)
        live = {'hopf_128_nngp': published_live(torch, g, 'hopf_128_nngp', 3565.0, 141),
                'fhn16_512_nngp_paged': published_live(torch, g, 'fhn16_512_nngp_paged', 17849.0, 517)}
        res['published_live'] = live
        res.update(published_runs(torch, g))
        res['published_k'] = published_k_table(torch, g, live)
        log('published K', json.dumps({k: (v['K'], v['published_K']) for k, v in res['published_k']['rows'].items()}))
        log('published runs', json.dumps({k: res[k]['wall_s'] for k in ('burgers_n128_published_schedule_nngp',
                                                                         'tomlab_n256_configs_schedule_nngp')}))
        res['gparareal_lorenz_n32'] = gparareal_lorenz(torch, g)
        res['gparareal_burgers_n128'] = gparareal_burgers(torch, g)
        res['gparareal_round_roofline'] = gpfull_round_roofline(torch, g)
        log('gparareal burgers', json.dumps(res['gparareal_burgers_n128']))
        log('gparareal lorenz K', res['gparareal_lorenz_n32']['K'], f"{res['gparareal_lorenz_n32']['wall_s']:.2f}s")
        res['burgers_n128_published_schedule'] = burgers_published_schedule(torch, g)
        res['tomlab_n256_published_schedule'] = tomlab_published_schedule(torch, g)
        res['hopf_n128_published_schedule'] = hopf_published_schedule(torch, g)
        res['tomlab_n256_published_schedule_contracted'] = tomlab_published_schedule(torch, g, fma=True)
        res['hopf_n128_published_schedule_contracted'] = hopf_published_schedule(torch, g, fma=True)
        res['fhn_pde_n512_fine_sweep'] = fhn_pde_fine_sweeps(torch, g)
        res['cpu_baseline'] = cpu_baseline(args.steps_per_slice, args.slices_per_gpu)
        res['cpu_nngp_corrections'] = cpu_corrections(res['nngp_correction_roofline'], res['cpu_baseline']['cores'])
        for v in res['nngp_correction_roofline'].values():
            v.pop('_preds', None)
        log('cpu corrections', json.dumps(res['cpu_nngp_corrections']))
        res['cpu_single_core'] = cpu_single_core()
        log('cpu single core', json.dumps(res['cpu_single_core']))
        # north-star target (>= 10x the CPU path on Burgers N=128, identical K): the CPU
        # restatement runs the same nnGParareal solve to convergence, measured (not extrapolated)
        c_s, c_f, c_r = burgers_cpu_converge(res['cpu_baseline']['cores'])
        g_r = runs['burgers']
        conv = res['burgers_n128_to_convergence']
        same = bool(np.array_equal(np.nan_to_num(g_r['u'], nan=7.0), np.nan_to_num(c_r['u'], nan=7.0)))
        res['burgers_n128_vs_cpu'] = {
            'gpu_to_convergence_s': conv['wall_s'], 'cpu_to_convergence_s': c_s,
            'speedup_to_convergence': c_s / conv['wall_s'], 'K_gpu': conv['K'], 'K_cpu': c_r['k'],
            'iterates_bitwise_equal': same, 'cpu_F_s': c_f, 'cpu_cores': res['cpu_baseline']['cores'],
            'host_cpus_total': os.cpu_count(), 'cpu_model': cpu_model(),
            'cores_note': f"the CPU solve ran {res['cpu_baseline']['cores']} OpenMP threads (this process's CPU "
                          f"affinity) of the {os.cpu_count()} CPUs the host reports; the ratio is against those "
                          f"threads, not the whole host",
            'note': 'CPU = oracle C restatement (gcc -O3 -march=x86-64-v4, OpenMP over slices and fits), '
                    'F in the reference dense formulation; the whole run to convergence on both sides'}
        log('burgers cpu', json.dumps(res['burgers_n128_vs_cpu']))
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
