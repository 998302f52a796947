"""Parareal driver -- the reference's Parareal(ode, solver, tspan, N, epsilon).run(model=...,
pool=..., parall=..., nn=..., seed=...) surface (parareal.py:26-471) with a device-resident loop.

Per iteration k (parareal.py:301-439):
  1. F over the unconverged slices [I, N): ONE nngp_rk_batch launch (replaces
     pool.map(solver.run_F_timed, ...) at :310-315).  With torch.distributed initialised and
     world_size > 1 the slices are split into contiguous blocks, one per rank/GPU, followed by a
     single all-gather of the fine end states (RCCL over xGMI) -- the only collective.
  2. training-set growth (:331-339) appended on the device (no host round trip).
  3. the SEQUENTIAL correction sweep i = I..N-1 (:359-382): G (one-slice nngp_rk_batch),
     model prediction (nngp_predict, or the classic F-G update), u[i+1] = preds + uG[i+1] -- all
     queued on one HIP stream without host synchronisation; the sweep is replicated on every rank
     (same inputs, same RNG draws), so ranks stay bit-identical without a broadcast.
  4. the slice errors ||u^{k+1} - u^k||_inf on the device, then ONE device->host copy per
     iteration (new iterate, coarse column, new D rows, errors) for the result dict and the
     convergence scan (:396-416), which advances I on the host exactly as the reference does.
The returned dict has the reference's keys ('t', 'u', 'err', 'x', 'D', 'k', 'data_x', 'data_D',
'timings', 'debug_dict', 'converged', 'conv_int').
"""
import ctypes
import json
import os
import time
import warnings

import numpy as np

from . import _lib
from .models import JITTERS, MAX_NEIGHBOURS, BareParareal, GPjax_p, NNGP_p
from .solver import SolverAbstr
from .systems import ODE


class MyPool():
    """Serial executor of the reference (parareal.py:16-24)."""

    @staticmethod
    def map(*args, chunksize=None, **kwargs):
        return map(*args, **kwargs)

    @staticmethod
    def shutdown(*args, **kwargs):
        pass


class GpuPool(MyPool):
    """Executor stand-in: the work the reference fans out through pool.map (fine solves, GP fits)
    is batched into single GPU launches by the driver and models, so the pool itself only has to
    provide the reference's map/shutdown surface."""


class _Events:
    def __init__(self, torch):
        self.torch = torch
        self.pairs = []

    def start(self):
        e = self.torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def stop(self, start, bucket):
        e = self.torch.cuda.Event(enable_timing=True)
        e.record()
        self.pairs.append((start, e, bucket))

    def collect(self):
        out = {}
        if self.pairs:
            self.pairs[-1][1].synchronize()   # stream-ordered: the last event completes last
        for a, b, k in self.pairs:
            out[k] = out.get(k, 0.0) + a.elapsed_time(b) / 1e3
        self.pairs = []
        return out


class _Ring:
    """Two-column stand-in for the [N+1][n][K] iterate history: PararealLight keeps only the
    current and next iterates (parareal.py:851-862), so u[..., k] addresses column k % 2."""

    def __init__(self, rows, n):
        self.a = np.full((rows, n, 2), np.nan)

    def __getitem__(self, key):
        i, j, k = key
        return self.a[i, j, k % 2]

    def __setitem__(self, key, v):
        i, j, k = key
        self.a[i, j, k % 2] = v


def shard_bounds(I, N, world, rank):
    """Contiguous block of the unconverged slices [I, N) owned by `rank`: every
    rank gets ceil((N-I)/world) slices (the last ones fewer or none), so one fixed-size all-gather
    reassembles them in slice order.  Returns (lo, hi, chunk)."""
    n_c = N - I
    chunk = (n_c + world - 1) // world
    lo = I + min(rank * chunk, n_c)
    hi = I + min((rank + 1) * chunk, n_c)
    return lo, hi, chunk


def native_comm_default():
    """The library's own RCCL communicator (include/nngp.h nngp_comm_*) for the collectives is
    opt-in -- run(..., native_comm=True) or NNGP_NATIVE_COMM=1 -- until a multi-GPU run has checked
    it bitwise against torch.distributed's (bench.py --gpus N records that check); by default the
    collectives are torch.distributed's (RCCL on an NCCL group)."""
    return os.environ.get('NNGP_NATIVE_COMM') == '1'


def fine_sweep_sharded(propagate, t, U, UF, I, N, group=None, native=None):
    """The fine sweep of one Parareal iteration, UF[I+1:N+1] = F(t[I:N], t[I+1:N+1], U[I:N])
    (parareal.py:310-327), sharded over the ranks of `group`: each rank integrates its contiguous
    block with ONE batched launch (`propagate(t0, t1, U0, out)`), then a single all-gather of the
    [chunk][d] end states (RCCL over xGMI; gloo on CPU) gives every rank the full result.  That
    all-gather is the only collective of the Parareal iteration.  native: use the library's
    communicator (nngp_allgather_states) instead of torch.distributed's (default
    native_comm_default())."""
    import torch
    dist = torch.distributed
    world = dist.get_world_size(group) if (dist.is_available() and dist.is_initialized()) else 1
    if world == 1:
        propagate(t[I:N], t[I + 1:N + 1], U[I:N], UF[I + 1:N + 1])
        return
    rank = dist.get_rank(group)
    lo, hi, chunk = shard_bounds(I, N, world, rank)
    n = U.shape[1]
    if dist.get_backend(group) == 'gloo':
        send = torch.zeros((chunk, n), dtype=U.dtype, device=U.device)
        if hi > lo:
            propagate(t[lo:hi], t[lo + 1:hi + 1], U[lo:hi].contiguous(), send[:hi - lo])
        gathered = _gloo_all_gather(send, group, world)
    else:
        # RCCL over xGMI: each rank integrates straight into its block of the gather buffer, then
        # ONE in-place all-gather -- the library's communicator (nngp_allgather_states) when live,
        # torch.distributed's otherwise
        gathered = torch.zeros((world * chunk, n), dtype=U.dtype, device=U.device)
        send = gathered[rank * chunk:(rank + 1) * chunk]
        if hi > lo:
            propagate(t[lo:hi], t[lo + 1:hi + 1], U[lo:hi].contiguous(), send[:hi - lo])
        if (native_comm_default() if native is None else native) and _lib.comm_for(group):
            _lib.check(_lib.lib().nngp_allgather_states(send.data_ptr(), gathered.data_ptr(), chunk * n,
                                                        torch.cuda.current_stream().cuda_stream))
        else:
            dist.all_gather_into_tensor(gathered, send, group=group)
    UF[I + 1:N + 1] = gathered[:N - I]


def _gloo_all_gather(send, group, world):
    """gloo's list all-gather; device tensors are staged through host memory (several ranks
    sharing one GPU, where RCCL refuses duplicate devices -- the multi-rank GPU tests)."""
    import torch
    host = send.detach().cpu()
    parts = [torch.empty_like(host) for _ in range(world)]
    torch.distributed.all_gather(parts, host, group=group)
    return torch.cat(parts).to(send.device)


def _all_gather_flat(send, group, world):
    """All-gather of equal-size 1-D/2-D blocks in rank order (RCCL all_gather_into_tensor, or
    the list form on gloo)."""
    import torch
    dist = torch.distributed
    if dist.get_backend(group) == 'gloo':
        return _gloo_all_gather(send, group, world)
    out = torch.empty((world * send.shape[0],) + tuple(send.shape[1:]), dtype=send.dtype, device=send.device)
    dist.all_gather_into_tensor(out, send, group=group)
    return out


def correction_sweep_sharded(coarse, predict_range, assemble, I, N, U1, UG1, d, group=None):
    """The sequential correction sweep (parareal.py:359-382) with each prediction's d*9*R fits
    sharded by coordinate over the ranks of `group` (worth it when d*9 is large,
    FHN-PDE d=800 has 7200 fits per prediction).  Per slice i: every rank runs the coarse step
    `coarse(i, U1[i], UG1[i+1])` (replicated, deterministic), its own coordinate block
    `predict_range(i, c0, c1, U1[i], out)`, ONE all-gather of the [chunk] predictions, and
    `assemble(preds[:d], UG1[i+1], U1[i+1])` (u = preds + uG).  Ranks stay bit-identical."""
    import torch
    dist = torch.distributed
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    c0, c1, chunk = shard_bounds(0, d, world, rank)
    send = torch.zeros(chunk, dtype=U1.dtype, device=U1.device)
    for i in range(I, N):
        coarse(i, U1[i], UG1[i + 1])
        if c1 > c0:
            predict_range(i, c0, c1, U1[i], send[:c1 - c0])
        preds = _all_gather_flat(send, group, world)
        assemble(preds[:d], UG1[i + 1], U1[i + 1])


class Parareal():
    _light = False

    def __init__(self, ode, solver, tspan, N, epsilon=5e-7, verbose='v', process_group=None, **kwargs):
        if not isinstance(ode, ODE):
            raise Exception('ode must be an instance of the ODE class, see systems.py file.')
        if not isinstance(solver, SolverAbstr):
            raise Exception('solver must be an instance of the SolverAbstr class, see solver.py file.')
        self.tspan = tspan
        self.N = N
        self.epsilon = epsilon
        self.runs = dict()
        self.fine = None
        self.ode_name = ode.name
        self.n = ode.get_dim()
        self.ode = ode
        self.solver = solver
        self.f = ode.get_vector_field()
        self.u0 = ode.get_init_cond()
        self.verbose = verbose
        self.process_group = process_group
        # nnGP sweep speculation (include/nngp.h nngp_correction_sweep): -1 auto, 0 off, 1 on
        self.speculate = int(kwargs.get('speculate', -1))
        self.shard_corrections = kwargs.get('shard_corrections')
        self.spec_hits = []

    def _get_pool(self, *args, **kwargs):
        pool = kwargs.get('pool', None)
        if pool is None or isinstance(pool, int):
            pool = GpuPool()   # no worker processes: the fan-outs are GPU launches
        return pool

    def run(self, *args, **kwargs):
        pool = self._get_pool(*args, **kwargs)
        kwargs['pool'] = pool
        try:
            out = self._run(*args, **kwargs)
        except Exception:
            pool.shutdown()
            raise
        pool.shutdown()
        return out

    def _run(self, model='parareal', cstm_mdl_name=None, add_model=False, **kwargs):
        if model.lower() == 'parareal':
            mdl = BareParareal(N=self.N, **kwargs)
        elif model.lower() == 'nngp':
            mdl = NNGP_p(n=self.n, N=self.N, worker_pool=kwargs['pool'], **kwargs)
            # nn='adaptive' grows m = k+2 (models.py:172-175); the GPU fits stop at m = 64, i.e. a
            # run still unconverged after 63 iterations raises there.  Say so before any work.
            es = kwargs.get('early_stop')
            k_last = min(self.N, es if es is not None else self.N) - 1
            if mdl.nn == 'adaptive' and max(10, k_last + 2) > MAX_NEIGHBOURS:
                warnings.warn(f"nn='adaptive' with N={self.N}: iteration {MAX_NEIGHBOURS - 1} would need "
                              f'm={MAX_NEIGHBOURS + 1} neighbours, beyond the GPU fits\' {MAX_NEIGHBOURS}; the run '
                              f'raises if it gets there (pass early_stop <= {MAX_NEIGHBOURS - 1} or a fixed nn)')
        elif model.lower() == 'gpjax':
            mdl = GPjax_p(n=self.n, N=self.N, worker_pool=kwargs['pool'], **kwargs)
            if 'process_group' not in kwargs:
                mdl.process_group = self.process_group   # the fits shard over the driver's group
        elif model.lower() == 'elm':
            raise NotImplementedError(f'model {model!r} is outside the GParareal/nnGP path (SURVEY.md §7)')
        else:
            raise Exception('Not implemented')
        s_time = time.time()
        out = self._parareal(mdl, **kwargs)
        elap_time = time.time() - s_time
        out['timings']['runtime'] = elap_time
        if self.verbose == 'v':
            print(f'Elapsed Parareal time: {elap_time:0.2f}s')
        if add_model:
            out['mdl'] = mdl.store()
        if cstm_mdl_name is None:
            cstm_mdl_name = mdl.name
        self.runs[cstm_mdl_name] = out
        return out

    # ------------------------------------------------------------------------ checkpoints
    def store(self, name, path='', mdl=None, objs=None):
        """Checkpoint (parareal.py:114-139).  The reference pickles the whole Parareal object;
        here the arrays go to `<path>/<name>.npz` and everything else (scalars, the model's
        settings, counters and its np.random.Generator state) to a JSON string inside it, so a
        checkpoint is loadable with numpy's safe loader (allow_pickle=False)."""
        if path and not os.path.exists(path):
            os.makedirs(path)
        arrays, meta = {}, {'format': 'nngp_amd-int-1', 'ode_name': self.ode_name, 'N': self.N,
                            'n': self.n, 'epsilon': self.epsilon, 'tspan': list(map(float, self.tspan))}
        for key, val in (objs or {}).items():
            if isinstance(val, np.ndarray):
                arrays[key] = val
            else:
                meta[key] = val.item() if isinstance(val, np.generic) else val
        if mdl is not None:
            meta['model'] = mdl.state_dict()
        arrays['meta'] = np.array(json.dumps(meta))
        np.savez(os.path.join(path, name + '.npz'), **arrays)

    @staticmethod
    def read_int_dump(file):
        """Load a store_int checkpoint written by `store` (numpy safe loader, no pickle)."""
        with np.load(file if file.endswith('.npz') else file + '.npz', allow_pickle=False) as z:
            state = {k: z[k] for k in z.files if k != 'meta'}
            state.update(json.loads(str(z['meta'])))
        return state

    def load_int_dump(self, other, cstm_mdl_name=None, add_model=False, **kwargs):
        """Resume a run from a store_int checkpoint (parareal.py:141-209): `other` is the
        checkpoint file (or its already-read state).  The model is rebuilt with its settings,
        counters and RNG state, so the resumed run draws exactly the stream it would have drawn."""
        state = other if isinstance(other, dict) else self.read_int_dump(other)
        if state['ode_name'] != self.ode_name or int(state['n']) != self.n or int(state['N']) != self.N:
            raise Exception('Input and previous ODEs do not match')
        mst = state['model']
        if mst['name'] == 'NNGP':
            mdl = NNGP_p(n=self.n, N=self.N, worker_pool=GpuPool(), **mst['settings'])
        elif mst['name'] == 'GP':
            mdl = GPjax_p(n=self.n, N=self.N, worker_pool=GpuPool(), **mst['settings'])
        else:
            mdl = BareParareal(N=self.N)
        mdl.load_state(mst)
        base_time = float(state['F_time']) + float(state['G_time']) + mdl.get_times()['mdl_tot_t']
        run_kwargs = dict(kwargs)
        run_kwargs.setdefault('pool', GpuPool())
        s_time = time.time()
        out = self._parareal(mdl, _resume=state, **run_kwargs)
        out['timings']['runtime'] = time.time() - s_time + base_time
        if add_model:
            out['mdl'] = mdl.store()
        self.runs[cstm_mdl_name or mdl.name] = out
        return out

    # ------------------------------------------------------------------------------ reports
    def _fine_reference(self):
        """The serial fine solve the reports compare against (parareal.py:636-643): run_F_timed
        over the whole span from u0, cached in self.fine / self.fine_t."""
        if self.fine is None:
            self.fine, self.fine_t = self.solver.run_F_timed(self.tspan[0], self.tspan[-1], self.u0)
        return self.fine_t

    def print_times(self, mdl_speedup=None, expected_fine=None):
        """Markdown table of K, G/F/model times, runtime and speed-up of every run in self.runs
        (parareal.py:636-694): speed-up against the serial fine solve, or -- with mdl_speedup =
        a run name -- model-time speed-up against that run; expected_fine adds the speed-up
        expected from the fine cost alone."""
        ref_mdl = self.runs[mdl_speedup]['timings']['mdl_tot_t'] if mdl_speedup in self.runs else None
        fine_t = None if ref_mdl is not None else self._fine_reference()
        keys = ['G_time', 'F_time', 'mdl_train_t', 'mdl_pred_t', 'mdl_tot_t', 'runtime']
        head = ['Model', 'K', 'G', 'F', 'Train', 'Pred', 'Mdl Tot', 'Overall',
                'Mdl Speedup' if ref_mdl is not None else 'Speedup']
        if expected_fine is not None:
            head.append('E[Speedup]')
        rows = [['Fine'] + ['-'] * 6 + (['-', '-'] if ref_mdl is not None else [f'{fine_t:.2e}', '1'])]
        if expected_fine is not None:
            rows[0].append('1')
        for name, v in self.runs.items():
            tm = v['timings']
            row = [name, str(v['k'])] + [f'{tm[k]:.2e}' for k in keys]
            row.append(f'{(ref_mdl / tm["mdl_tot_t"]) if ref_mdl is not None else (fine_t / tm["runtime"]):.2f}')
            if expected_fine is not None:
                row.append(f'{expected_fine / (expected_fine / self.N * v["k"] + tm["mdl_tot_t"]):.2f}')
            rows.append(row)
        width = [max(len(r[i]) for r in [head] + rows) for i in range(len(head))]
        line = lambda r: '|' + '|'.join(f'{x:^{w}}' for x, w in zip(r, width)) + '|'
        out = '\n'.join([line(head), '|' + '|'.join('-' * w for w in width) + '|'] + [line(r) for r in rows])
        print(out)
        return out

    def print_speedup(self, mdls=None, md=True, fine_t=None, F_t=None, mdl_title=''):
        """Speed-up table (parareal.py:697-758), markdown (md=True) or a LaTeX tabular: per run
        K, G and F time per iteration, model time, total and speed-up against fine_t (or the
        cached serial fine solve); with F_t, the total is modelled as F_t*K + model time."""
        sep, beg, end = (' | ', '|', '|') if md else (' & ', '', '\\\\')
        Fh, Gh = ('F', 'G') if md else ('$T_{\\f}$', '$T_{\\g}$')
        if F_t is not None:
            fine_t = F_t * self.N
        if fine_t is None:
            fine_t = self.fine_t if self.fine is not None else None
        if fine_t is None:
            raise Exception('Running time of fine solver unknown/not provided')
        names = {'GP': 'GParareal', 'NNGP': 'NN-GParareal'}
        tab = [['Model', 'K', Gh, Fh, 'Model', 'Total', 'Speed-up'],
               ['---'] * 7 if md else ['\\hline'],
               ['Fine', '-', '-', '-', '-', f'{fine_t:.2e}', '1']]
        for key, label in (mdls if mdls is not None else {k: k for k in self.runs}).items():
            if key not in self.runs:
                raise Exception('Unknown model', key)
            r = self.runs[key]
            tm = r['timings']
            total = F_t * r['k'] + tm['mdl_tot_t'] if F_t is not None else tm['runtime']
            tab.append([names.get(label, label), str(r['k']), f'{tm["G_time"] / r["k"]:.2e}',
                        f'{tm["F_time"] / r["k"]:.2e}', f'{tm["mdl_tot_t"]:.2e}', f'{tm["runtime"]:.2e}',
                        f'{fine_t / total:.2f}'])
        lines = [beg + sep.join(r) + end for r in tab]
        if md:
            lines = [f'$N={self.N}$\n'] + lines
        else:
            lines = ([r'\caption*{' + mdl_title + r', $N=' + f'{self.N}' + r'$}', r'\begin{tabular}{lcccccc}']
                     + lines + [r'\end{tabular}\\    \bigskip' + '\n'])
        out = '\n'.join(lines)
        print(out)
        return out

    # ------------------------------------------------------------------------------ F sweep
    def _fine_sweep(self, torch, t_dev, Uk, UF, I, N, n):
        """uF[I+1:N+1] = F(u[I:N]) -- sharded over ranks when a process group is active."""
        fine_sweep_sharded(lambda a, b, u, out: self.solver.run_F_batch(a, b, u, out=out),
                           t_dev, Uk, UF, I, N, self.process_group, native=self._run_native_comm)

    # ------------------------------------------------------------------ correction sweep
    def _correction_sweep(self, torch, model, t_dev, I, N, U1, UG1, UF, UG, X, Y, rows, th0, stream):
        """The sequential sweep i = I..N-1 of parareal.py:359-382 (G, correction, u = preds + uG)
        as ONE native call (nngp_correction_sweep) that queues every slice's launches back to back.
        Returns the device time of the G launches in seconds."""
        solver, lib = self.solver, _lib.lib()
        if N <= I:
            return 0.0
        if solver.coarse_is_paged():   # paged coarse solve (never in the reference configs)
            return self._correction_sweep_py(torch, model, t_dev, I, N, U1, UG1, UF, UG, X, Y, rows,
                                             th0, stream)
        cs = solver.f.csystem(U1.device)
        g_ms = ctypes.c_float(0.0)
        if isinstance(model, NNGP_p) and self._shard_corrections(model):
            return self._correction_sweep_sharded(torch, model, t_dev, I, N, U1, UG1, X, Y, rows, th0, stream)
        if isinstance(model, NNGP_p):
            m = min(model.n_neighbours(), int(rows))
            jit, jp = _lib.host_doubles(JITTERS)
            if not hasattr(self, '_preds_scratch') or self._preds_scratch.device != U1.device:
                self._preds_scratch = torch.empty(self.n, dtype=torch.float64, device=U1.device)
            hits = ctypes.c_int32(0)
            # auto speculation (-1): after an iteration whose guesses hit fewer than 5 % of its
            # slices (a chaotic field: TomLab N = 256 hits 1-3 of ~250), the next 7 iterations run
            # without the speculative batch and re-speculation -- their side-stream fits only
            # compete with the sweep's own (TomLab 3.54 -> 2.64 s over 20 iterations) -- then it is
            # tried again.  The fits, hence every iterate, are the same either way.
            spec = self._run_speculate
            if spec < 0 and getattr(self, '_spec_skip', 0) > 0:
                self._spec_skip -= 1
                spec = 0
            _lib.check(lib.nngp_correction_sweep(
                ctypes.byref(cs), _lib.TABLEAU[solver.G], solver.step_mode, solver.Ng, t_dev.data_ptr(), I, N,
                U1.data_ptr(), UG1.data_ptr(), UF.data_ptr(), UG.data_ptr(), _lib.MODEL_NNGP, X.data_ptr(),
                Y.data_ptr(), int(rows), m, len(jit), jp, model.n_restarts, th0.data_ptr(), float(model.fatol),
                float(model.xatol), model.maxfev, self._preds_scratch.data_ptr(), spec,
                ctypes.byref(hits), ctypes.byref(g_ms), stream))
            model.train_count += model.n_fits * (N - I)
            self.spec_hits.append(int(hits.value))
            if spec < 0 and N - I >= 2 and hits.value < 0.05 * (N - I):
                self._spec_skip = 7
        elif isinstance(model, GPjax_p):
            Xg, alpha, coef = model._dev
            _lib.check(lib.nngp_correction_sweep(
                ctypes.byref(cs), _lib.TABLEAU[solver.G], solver.step_mode, solver.Ng, t_dev.data_ptr(), I, N,
                U1.data_ptr(), UG1.data_ptr(), UF.data_ptr(), UG.data_ptr(), _lib.MODEL_GPFULL, Xg.data_ptr(),
                alpha.data_ptr(), Xg.shape[0], 0, 0, None, 0, coef.data_ptr(), 0.0, 0.0, 0, None, 0, None,
                ctypes.byref(g_ms), stream))
        else:
            _lib.check(lib.nngp_correction_sweep(
                ctypes.byref(cs), _lib.TABLEAU[solver.G], solver.step_mode, solver.Ng, t_dev.data_ptr(), I, N,
                U1.data_ptr(), UG1.data_ptr(), UF.data_ptr(), UG.data_ptr(), _lib.MODEL_PARAREAL, None, None,
                0, 0, 0, None, 0, None, 0.0, 0.0, 0, None, 0, None, ctypes.byref(g_ms), stream))
        return g_ms.value / 1e3

    def _shard_corrections(self, model):
        """Shard each prediction's fits by coordinate over the process group: Parareal(...,
        shard_corrections=True/False) or run(..., shard_corrections=...) for one run (True applies
        at any world size, one rank included); by default when more than one rank and
        d*9*R >= 2048."""
        import torch
        dist = torch.distributed
        if not (dist.is_available() and dist.is_initialized()):
            return False
        shard = getattr(self, '_run_shard', self.shard_corrections)
        if shard is not None:
            return bool(shard)
        return dist.get_world_size(self.process_group) > 1 and model.n_fits >= 2048

    def _correction_sweep_sharded(self, torch, model, t_dev, I, N, U1, UG1, X, Y, rows, th0, stream):
        """correction_sweep_sharded with the HIP launches.  On an NCCL group with the library's
        communicator live (and native_comm, opt-in: native_comm_default()): ONE native call,
        nngp_correction_sweep_sharded, that issues every slice's G, this rank's coordinates, the
        RCCL all-gather of the predictions and u = preds + uG on the stream with no host round trip.
        Otherwise (gloo: ranks sharing one GPU) the same launches from Python: G via the solver,
        nngp_predict_range for this rank's coordinates, u = (preds - 0) + uG via
        nngp_parareal_update (bitwise the fused kernel's mean + uG)."""
        lib, solver, n = _lib.lib(), self.solver, self.n
        m = min(model.n_neighbours(), int(rows))
        jit, jp = _lib.host_doubles(JITTERS)
        nf = model.n_fits
        if getattr(self, '_run_native_comm', False) and _lib.comm_for(self.process_group) and \
                not solver.coarse_is_paged():
            world = torch.distributed.get_world_size(self.process_group)
            # NNGP_SHARD_EMULATE_RANKS=W on one rank: this process plays the W ranks of the split
            # (include/nngp.h nngp_correction_sweep_sharded_emulated, a one-GPU check)
            emulate = max(1, int(os.environ.get('NNGP_SHARD_EMULATE_RANKS', '1'))) if world == 1 else 0
            vr = emulate or world
            chunk = (n + vr - 1) // vr
            gather = torch.zeros(vr * chunk, dtype=torch.float64, device=U1.device)
            cs = solver.f.csystem(U1.device)
            g_ms = ctypes.c_float(0.0)
            args = (ctypes.byref(cs), _lib.TABLEAU[solver.G], solver.step_mode, solver.Ng, t_dev.data_ptr(), I, N,
                    U1.data_ptr(), UG1.data_ptr(), X.data_ptr(), Y.data_ptr(), int(rows), m, len(jit), jp,
                    model.n_restarts, th0.data_ptr(), float(model.fatol), float(model.xatol), model.maxfev,
                    gather.data_ptr())
            if emulate:
                _lib.check(lib.nngp_correction_sweep_sharded_emulated(*args, gather.numel(), emulate,
                                                                      ctypes.byref(g_ms), stream))
            else:
                _lib.check(lib.nngp_correction_sweep_sharded(*args, ctypes.byref(g_ms), stream))
            model.train_count += nf * (N - I)
            self.spec_hits.append(0)
            return g_ms.value / 1e3
        zeros = torch.zeros(n, dtype=torch.float64, device=U1.device)
        ev = _Events(torch)

        def coarse(i, u, out):
            eg = ev.start()
            solver.run_G_batch(t_dev[i:i + 1], t_dev[i + 1:i + 2], u.view(1, -1), out=out.view(1, -1))
            ev.stop(eg, 'G')

        def predict_range(i, c0, c1, u, out):
            j = i - I
            _lib.check(lib.nngp_predict_range(
                X.data_ptr(), Y.data_ptr(), int(rows), n, u.data_ptr(), m, len(jit), jp, model.n_restarts,
                th0[j * nf:(j + 1) * nf].data_ptr(), c0, c1, float(model.fatol), float(model.xatol), model.maxfev,
                out.data_ptr(), stream))

        def assemble(preds, ug, out):
            _lib.check(lib.nngp_parareal_update(n, preds.data_ptr(), zeros.data_ptr(), ug.data_ptr(),
                                                out.data_ptr(), stream))

        correction_sweep_sharded(coarse, predict_range, assemble, I, N, U1, UG1, n, self.process_group)
        model.train_count += nf * (N - I)
        self.spec_hits.append(0)
        return ev.collect().get('G', 0.0)

    def _correction_sweep_debug(self, torch, model, t_dev, I, N, U1, UG1, UF, UG, X, Y, rows, th0, stream):
        """debug=True (parareal.py:353-392): the same per-slice sweep, keeping every prediction,
        then the 'truth' F(u[i]) - uG_new[i+1] for all slices at once -- ONE batched fine launch
        instead of the reference's N-I serial run_F calls -- and |truth - preds| per slice and
        coordinate.  Returns (G seconds, pred_err [N-I][n])."""
        lib, n = _lib.lib(), self.n
        P = torch.empty((N - I, n), dtype=torch.float64, device=U1.device)
        zeros = torch.zeros(n, dtype=torch.float64, device=U1.device)
        ev = _Events(torch)
        nf = model.n_fits if isinstance(model, NNGP_p) else 0
        for i in range(I, N):
            j = i - I
            eg = ev.start()
            self.solver.run_G_batch(t_dev[i:i + 1], t_dev[i + 1:i + 2], U1[i:i + 1], out=UG1[i + 1:i + 2])
            ev.stop(eg, 'G')
            if isinstance(model, NNGP_p):
                model.predict_device(X, Y, rows, U1[i], th0[j * nf:(j + 1) * nf], out=U1[i + 1],
                                     bias=UG1[i + 1], preds=P[j], stream=stream)
            else:
                if isinstance(model, GPjax_p):
                    model.predict_device(U1[i], out=P[j], stream=stream)
                else:   # BareParareal: uF - uG (models.py:82-83)
                    _lib.check(lib.nngp_parareal_update(n, UF[i + 1].data_ptr(), UG[i + 1].data_ptr(), None,
                                                        P[j].data_ptr(), stream))
                _lib.check(lib.nngp_parareal_update(n, P[j].data_ptr(), zeros.data_ptr(), UG1[i + 1].data_ptr(),
                                                    U1[i + 1].data_ptr(), stream))
        truth = torch.empty((N - I, n), dtype=torch.float64, device=U1.device)
        self.solver.run_F_batch(t_dev[I:N], t_dev[I + 1:N + 1], U1[I:N].contiguous(), out=truth)
        _lib.check(lib.nngp_parareal_update((N - I) * n, truth.data_ptr(), UG1[I + 1:N + 1].data_ptr(), None,
                                            truth.data_ptr(), stream))
        pred_err = np.abs(truth.cpu().numpy() - P.cpu().numpy())
        return ev.collect().get('G', 0.0), pred_err

    def _correction_sweep_py(self, torch, model, t_dev, I, N, U1, UG1, UF, UG, X, Y, rows, th0, stream):
        """Per-slice Python loop (paged coarse solver only): same launches, issued one by one."""
        lib = _lib.lib()
        ev = _Events(torch)
        nf = model.n_fits if isinstance(model, NNGP_p) else 0
        for i in range(I, N):
            eg = ev.start()
            self.solver.run_G_batch(t_dev[i:i + 1], t_dev[i + 1:i + 2], U1[i:i + 1], out=UG1[i + 1:i + 2])
            ev.stop(eg, 'G')
            if isinstance(model, NNGP_p):
                j = i - I
                model.predict_device(X, Y, rows, U1[i], th0[j * nf:(j + 1) * nf], out=U1[i + 1],
                                     bias=UG1[i + 1], stream=stream)
            elif isinstance(model, GPjax_p):
                model.predict_device(U1[i], out=U1[i + 1], bias=UG1[i + 1], stream=stream)
            else:   # (uF - uG_prev) + uG_new   (models.py:82-83, parareal.py:382)
                _lib.check(lib.nngp_parareal_update(self.n, UF[i + 1].data_ptr(), UG[i + 1].data_ptr(),
                                                    UG1[i + 1].data_ptr(), U1[i + 1].data_ptr(), stream))
        return ev.collect().get('G', 0.0)

    # --------------------------------------------------------------------------- main loop
    def _parareal(self, model, debug=False, early_stop=None, parall='Serial', store_int=False,
                  _resume=None, **kwargs):
        torch = _lib.require_gpu()
        light = self._light
        if light:   # PararealLight (parareal.py:812-1060)
            if debug:
                print('WARNING: PararealLight does not support debug mode')
                debug = False
            if store_int:
                raise NotImplementedError('PararealLight does not support storing intermediate results')
            if kwargs.get('lag_k') is not None or _resume is not None:
                raise NotImplementedError('PararealLight keeps no per-iteration training history')
        if debug and self.process_group is not None:
            raise NotImplementedError('debug mode runs on one rank')
        one_step_error, all_pred_err = [], []   # debug (parareal.py:258-262)
        self.spec_hits = []
        # run(..., speculate=, shard_corrections=) override the constructor's settings for this run
        self._run_speculate = int(kwargs.get('speculate', self.speculate))
        self._spec_skip = 0   # auto speculation: iterations left to run without it (_correction_sweep)
        self._run_shard = kwargs.get('shard_corrections', self.shard_corrections)
        self._run_native_comm = bool(kwargs.get('native_comm', native_comm_default()))
        tspan, N, epsilon, n = self.tspan, self.N, self.epsilon, self.n
        solver = self.solver
        verbose = kwargs.get('verbose', self.verbose)
        dev = torch.device('cuda', torch.cuda.current_device())
        f64 = dict(dtype=torch.float64, device=dev)
        lib = _lib.lib()
        stream = torch.cuda.current_stream().cuda_stream
        ev = _Events(torch)
        is_nngp = isinstance(model, NNGP_p)

        t = np.linspace(tspan[0], tspan[1], num=N + 1)
        t_dev = torch.tensor(t, **f64)
        I = 0
        conv_int = []
        # The iterate history [N+1][n][k] and data_x / data_D [N][n][k] (parareal.py:233-246) hold
        # one column per iteration.  They are allocated for 16 iterations and doubled when a run
        # needs more: the reference's np.empty((N+1, n, N+1)) is 1.7 GB each at FHN-PDE d = 800,
        # N = 512, whose runs converge in K = 2.  The returned slices [..., :k+1] are the same values.
        cap0 = min(N + 1, 16)
        u = _Ring(N + 1, n) if light else np.full((N + 1, n, cap0), np.nan)
        err = np.full((N + 1, N), np.nan)
        x = np.zeros((0, n))
        D = np.zeros((0, n))
        data_x = None if light else np.full((N, n, cap0), np.nan)
        data_D = None if light else np.full((N, n, cap0), np.nan)

        def ensure_cols(c):   # history columns 0 .. c-1 exist
            nonlocal u, data_x, data_D
            if light or u.shape[2] >= c:
                return
            cap = min(N + 1, max(c, 2 * u.shape[2]))

            def grown(a):
                b = np.full(a.shape[:2] + (cap,), np.nan)
                b[..., :a.shape[2]] = a
                return b
            u, data_x, data_D = grown(u), grown(data_x), grown(data_D)
        last = 0   # the column of u holding the newest iterate
        G_time = F_time = F_time_serial = 0.0

        u0 = torch.tensor(self.u0, **f64)
        Uk = torch.empty((N + 1, n), **f64)
        UGk = torch.empty((N + 1, n), **f64)
        UF = torch.empty((N + 1, n), **f64)
        UGk[0] = u0
        UF[0] = u0
        if _resume is None:
            # initial coarse sweep, sequential (parareal.py:265-270; legacy: one global grid,
            # new_lib.py:902-906 -- the solver decides)
            e0 = ev.start()
            solver.initial_coarse(t_dev, UGk, N)
            ev.stop(e0, 'G')
            Uk.copy_(UGk)
            u[:, :, 0] = Uk.cpu().numpy()
            G_time += ev.collect().get('G', 0.0)
            k_start = 0
        else:   # continue from a store_int checkpoint (parareal.py:141-209, 279-297)
            kc = int(_resume['k'])
            I, conv_int = int(_resume['I']), [int(c) for c in _resume['conv_int']]
            ensure_cols(kc + 2)
            u[:, :, :kc + 2] = _resume['u']
            err[:, :kc + 1] = _resume['err']
            x, D = np.array(_resume['x']), np.array(_resume['D'])
            data_x[..., :kc + 1] = _resume['data_x']
            data_D[..., :kc + 1] = _resume['data_D']
            G_time, F_time = float(_resume['G_time']), float(_resume['F_time'])
            F_time_serial = float(_resume['F_time_serial'])
            Uk.copy_(torch.tensor(u[:, :, kc + 1], **f64))
            UGk.copy_(torch.tensor(_resume['uG_cur'], **f64))
            k_start = kc + 1
            if I == N:   # parareal.py:294-295
                raise Exception('System has already converged')

        cap = max(4 * N, 64, 2 * x.shape[0])
        Xd = torch.empty((cap, n), **f64)
        Dd = torch.empty((cap, n), **f64)
        rows = x.shape[0]
        if rows:
            Xd[:rows] = torch.tensor(x, **f64)
            Dd[:rows] = torch.tensor(D, **f64)
        k = k_start
        th_pin = None   # pinned host staging of the initial-theta draws (async upload)
        for k in range(k_start, N):
            ensure_cols(k + 2)   # this iteration writes u[..., k + 1] and data_x / data_D[..., k]
            if verbose == 'v':
                print(f'{self.ode_name} {model.name} iteration number (out of {N}): {k + 1} ')
            e0 = ev.start()
            self._fine_sweep(torch, t_dev, Uk, UF, I, N, n)
            ev.stop(e0, 'F')
            n_F = N - I                       # slices of this iteration's fine sweep
            Uk1 = Uk.clone()
            UGk1 = UGk.clone()
            Uk1[I + 1] = UF[I + 1]            # u[I+1,:,k+1:] = uF[I+1,:,k]   (:331-333)
            I = I + 1
            # training data (:336-339): x += u[I-1:N,:,k]; D += uF[I:N+1,:,k] - uG[I:N+1,:,k].
            # Appended on the device; the host copy of the new D rows travels with the iteration's
            # single device->host copy below (no host round trip between F and the sweep).
            new = N + 1 - I
            if rows + new > Xd.shape[0]:
                grow = max(2 * Xd.shape[0], rows + new)
                Xd = torch.cat([Xd[:rows], torch.empty((grow - rows, n), **f64)])
                Dd = torch.cat([Dd[:rows], torch.empty((grow - rows, n), **f64)])
            Xd[rows:rows + new] = Uk[I - 1:N]
            _lib.check(lib.nngp_parareal_update(new * n, UF[I:N + 1].data_ptr(), UGk[I:N + 1].data_ptr(),
                                                None, Dd[rows:rows + new].data_ptr(), stream))
            rows += new
            x = np.vstack([x, u[I - 1:N, :, k]])
            if not light:
                data_x[I - 1:N, :, k] = u[I - 1:N, :, k]

            def take_D(d_new):
                nonlocal D
                D = np.vstack([D, d_new])
                if not light:
                    data_D[I - 1:N, :, k] = d_new

            if I == N:                          # early stop (:343-348)
                if verbose == 'v':
                    print('WARNING: early stopping')
                take_D(Dd[rows - new:rows].cpu().numpy())
                u[:, :, k + 1] = Uk1.cpu().numpy()
                err[:, k] = np.linalg.norm(u[:, :, k + 1] - u[:, :, k], np.inf, 1)
                last = k if light else k + 1   # PararealLight returns u_curr here
                err[-1, k] = np.nextafter(epsilon, 0)
                fe = ev.collect()
                F_time += fe.get('F', 0.0)
                F_time_serial += fe.get('F', 0.0)
                break

            lag_k = kwargs.get('lag_k')
            d_pending = True
            if lag_k is None:
                # the models train on the device-resident set (fit stores it; no host copy)
                model.fit_timed(Xd[:rows], Dd[:rows], k=k, data_x=data_x, data_y=data_D)
                Xs, Ds, rows_s = Xd, Dd, rows
            else:   # legacy: train on the last lag_k iterations only (new_lib.py:980-987)
                take_D(Dd[rows - new:rows].cpu().numpy())
                d_pending = False
                tr_x = np.moveaxis(data_x[I:, :, max(k + 1 - lag_k, 0):k + 1], 1, -1).reshape(-1, n)
                tr_y = np.moveaxis(data_D[I:, :, max(k + 1 - lag_k, 0):k + 1], 1, -1).reshape(-1, n)
                model.fit_timed(tr_x, tr_y, k=k)
                Xs, Ds, rows_s = torch.tensor(tr_x, **f64), torch.tensor(tr_y, **f64), tr_x.shape[0]
            if is_nngp:
                draws = torch.from_numpy(model.draw_thetas(N - I))
                if th_pin is None or th_pin.numel() < draws.numel():
                    th_pin = torch.empty(max(draws.numel(), 2 * N * model.n_fits), dtype=torch.float64,
                                         pin_memory=True)
                # the previous iteration's upload finished before its host copy below returned
                th_pin[:draws.numel()].copy_(draws.view(-1))
                th0 = torch.empty(draws.shape, **f64)
                th0.view(-1).copy_(th_pin[:draws.numel()], non_blocking=True)
            e_loop = ev.start()
            if debug:
                g_s, pred_err = self._correction_sweep_debug(torch, model, t_dev, I, N, Uk1, UGk1, UF, UGk, Xs, Ds,
                                                             rows_s, th0 if is_nngp else None, stream)
                if verbose == 'v':
                    print(f'Avg error {np.mean(pred_err, 0)}, Max. error {np.max(pred_err, 0)}')
                all_pred_err.append(pred_err)
            else:
                g_s = self._correction_sweep(torch, model, t_dev, I, N, Uk1, UGk1, UF, UGk, Xs, Ds, rows_s,
                                             th0 if is_nngp else None, stream)
            ev.stop(e_loop, 'loop')
            # ONE device->host copy per iteration: the new iterate (the reference's u[:, :, k+1]),
            # the new coarse column (NaN guard, checkpoint), the new D rows and the slice errors
            # ||u^{k+1}_p - u^k_p||_inf (parareal.py:402-403; torch.amax propagates NaN as np.max).
            errk = torch.amax(torch.abs(Uk1 - Uk), dim=1)
            parts = [Uk1.reshape(-1), UGk1.reshape(-1), errk]
            if d_pending:
                parts.append(Dd[rows - new:rows].reshape(-1))
            host = torch.cat(parts).cpu().numpy()
            sz = (N + 1) * n
            u[:, :, k + 1] = host[:sz].reshape(N + 1, n)
            last = k + 1
            ug = host[sz:2 * sz].reshape(N + 1, n)
            if d_pending:
                take_D(host[2 * sz + N + 1:].reshape(new, n))
            te = ev.collect()
            F_time += te.get('F', 0.0)
            # F_time_serial_avg (parareal.py:314): the per-slice fine time averaged over the
            # iteration's slices.  Every slice of the batched launch runs from its start to its end
            # (a lone slice takes as long: the chain of steps is the cost), so each slice's time is
            # the launch's and so is their mean.
            F_time_serial += te.get('F', 0.0) if n_F > 0 else 0.0
            G_time += g_s
            model.add_pred_time(max(te.get('loop', 0.0) - g_s, 0.0))
            if np.any(np.isnan(ug)):
                raise Exception('NaN values in initial coarse solve - increase Ng!')
            err[:, k] = host[2 * sz:2 * sz + N + 1]                                # (:402-403)
            err[I, k] = 0
            if debug:   # (:405-406)
                one_step_error.append([err[I + 1, k], pred_err.max()])
            II = I
            for p in range(II + 1, N + 1):                                          # (:408-416)
                if err[p, k] < epsilon:
                    I = I + 1
                else:
                    break
            if verbose == 'v':
                print('--> Converged:', I)
            conv_int.append(I)
            Uk, UGk = Uk1, UGk1
            if store_int:   # parareal.py:420-431 (npz + JSON instead of a pickle of the object)
                name_base = kwargs.get('int_name', f'{self.ode_name}_{self.N}_{model.name}_int')
                objs = {'t': t, 'I': I, 'k': k, 'conv_int': np.array(conv_int), 'u': u[..., :k + 2],
                        'uG_cur': ug, 'err': err[:, :k + 1], 'x': x, 'D': D, 'data_x': data_x[..., :k + 1],
                        'data_D': data_D[..., :k + 1], 'G_time': G_time, 'F_time': F_time,
                        'F_time_serial': F_time_serial, 'epsilon': epsilon, 'N': N,
                        'ode_name': self.ode_name}
                # <int_dir>/<name_base>/<name_base>_<k>.npz, the reference's layout (parareal.py:422-431)
                self.store(name=f'{name_base}_{k}', path=os.path.join(kwargs.get('int_dir', ''), name_base),
                           mdl=model, objs=objs)
            if I == N:
                break
            if (early_stop is not None) and k == (early_stop - 1):
                if verbose == 'v':
                    print('Early stopping due to user condition.')
                break
            # not in the reference: a wall-clock deadline (time.time() value) for runs longer than
            # one session, resumed later from their store_int dump (tools/published_k_run.py)
            if kwargs.get('stop_at') is not None and time.time() > kwargs['stop_at']:
                if verbose == 'v':
                    print('Stopping at the stop_at deadline; resume from the store_int dump.')
                break

        timings = {'F_time': F_time, 'G_time': G_time, 'F_time_serial_avg': F_time_serial,
                   'spec_hits': list(self.spec_hits)}
        timings.update(model.get_times())
        debug_dict = {}
        if debug:   # (:441-463; the reference also plots these)
            debug_dict = {'one_step_error': np.array(one_step_error), 'all_pred_err': all_pred_err}
        if light:   # (parareal.py:1057-1059): the newest iterate only, no data_x/data_D
            return {'t': t, 'u': u[:, :, last].copy(), 'err': err[:, :k + 1], 'x': x, 'D': D, 'k': k + 1,
                    'timings': timings, 'debug_dict': {}, 'converged': I == N, 'conv_int': conv_int}
        return {'t': t, 'u': u[:, :, :k + 1], 'err': err[:, :k + 1], 'x': x, 'D': D, 'k': k + 1,
                'data_x': data_x[..., :k + 1], 'data_D': data_D[..., :k + 1], 'timings': timings,
                'debug_dict': debug_dict, 'converged': I == N, 'conv_int': conv_int}


class PararealLight(Parareal):
    """parareal.py:812-1060: the same iteration keeping only the current and next iterates on the
    host (no [N+1][n][K] history, no per-iteration training arrays); returns the newest iterate
    as 'u'.  Checkpoints, plots and report tables are not supported, as in the reference."""
    _light = True

    def load_int_dump(self, *args, **kwargs):
        raise NotImplementedError('PararealLight does not support loading from intermediate dumps')

    def _run_from_int(self, *args, **kwargs):
        raise NotImplementedError('PararealLight does not support loading from intermediate dumps')

    def print_times(self, *args, **kwargs):
        raise NotImplementedError('PararealLight does not support printing times')

    def print_speedup(self, *args, **kwargs):
        raise NotImplementedError('PararealLight does not support printing speedup')
