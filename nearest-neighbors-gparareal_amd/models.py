"""Correction models -- the reference's ModelAbstr / BareParareal / NNGP_p plugin surface
(models.py:19-270) with the nearest-neighbour GP running on the GPU.

NNGP_p keeps the reference's constructor arguments (n, N, worker_pool, theta, fatol, xatol, nn,
seed, n_restarts, ...), its RNG (np.random.default_rng(seed), models.py:114) and the exact order
of its draws: per prediction, rng.integers(-8, 0, 2) once for every (coordinate, jitter,
restart) in itertools.product order (models.py:186-192).  A single vectorised
rng.integers(-8, 0, (count, 2)) yields the same stream (the range is a power of two, so
numpy's Lemire sampler never rejects; pinned by tests/test_host.py against tests/golden/rng.npz).

Compute paths (all HIP, no CPU fallback):
  predict(...)         reference signature, host arrays in/out -> nngp_predict (fused kernels)
  predict_device(...)  device tensors, used by the Parareal driver's sequential loop
  get_preds(...)       reference signature on pre-selected (xm, ym) -> nngp_nm_fit_batch +
                       first-argmin + nngp_gp_mean (the unfused path of the same kernels)

GPjax_p (models.py:273-473) is the full-data GParareal model: per coordinate and jitter a
Nelder-Mead fit of the GP over ALL training rows, warm-started at the previous optimum, batched
across fits on the GPU (nngp_gpfull_fit), and posterior means from the memoised Cholesky weights
(nngp_gpfull_mean / the native sweep).
"""
import copy
import ctypes
import time
from itertools import product

import numpy as np

from . import _lib

JITTERS = np.arange(-20, -11, dtype=float)   # models.py:186
MAX_NEIGHBOURS = 64   # the HIP fits' largest padded kernel size (include/nngp.h)


class ModelAbstr():

    def __init__(self, **kwargs):
        self.train_time = 0
        self.pred_time = 0
        N = kwargs['N']
        self.pred_times = np.zeros(N)
        self.time_k = 0

    def fit_timed(self, x, y, *args, **kwargs):
        self.time_k = kwargs['k']
        s_time = time.time()
        ret = self.fit(x, y, *args, **kwargs)
        elap_time = time.time() - s_time
        self.train_time += elap_time
        self.pred_times[self.time_k] += elap_time
        return ret

    def predict_timed(self, new_x, *args, **kwargs):
        s_time = time.time()
        ret = self.predict(new_x, *args, **kwargs)
        elap_time = time.time() - s_time
        self.pred_time += elap_time
        self.pred_times[self.time_k] += elap_time
        return ret

    def add_pred_time(self, seconds):
        """Device-measured prediction time (the Parareal driver times whole sweeps with events)."""
        self.pred_time += seconds
        self.pred_times[self.time_k] += seconds

    def get_times(self):
        return {'mdl_train_t': self.train_time, 'mdl_pred_t': self.pred_time,
                'mdl_tot_t': self.train_time + self.pred_time, 'by_iter': self.pred_times[:self.time_k + 1]}

    def fit(self, x, y, *args, **kwargs):
        self.x, self.y = x, y
        raise Exception('Not implemented')

    def predict(self, new_x, prev_F, prev_G):
        raise Exception('Not implemented')

    def state_dict(self):
        """Counters for a store_int checkpoint (JSON-serialisable)."""
        return {'name': self.name, 'train_time': self.train_time, 'pred_time': self.pred_time,
                'pred_times': self.pred_times.tolist(), 'time_k': self.time_k, 'settings': {}}

    def load_state(self, st):
        self.train_time, self.pred_time = st['train_time'], st['pred_time']
        self.pred_times = np.array(st['pred_times'], dtype=float)
        self.time_k = st['time_k']

    def store(self):
        if hasattr(self, 'pool'):
            pool = self.pool
            self.pool = None
            new = copy.deepcopy(self)
            self.pool = pool
        else:
            new = copy.deepcopy(self)
        return new


class BareParareal(ModelAbstr):
    """Classic Parareal correction F - G (models.py:74-83)."""

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.name = 'Parareal'

    def fit(self, *args, **kwargs):
        pass

    def predict(self, new_x, prev_F, prev_G, *args, **kwargs):
        return prev_F - prev_G


class NNGP_p(ModelAbstr):
    """Nearest-neighbour GP correction (models.py:98-270) on the GPU."""

    def __init__(self, n, N, worker_pool=None, theta=None, fatol=None, xatol=None, **kwargs):
        super().__init__(N=N, **kwargs)
        if theta is None:
            theta = [1, 1]
        self.theta = np.array(theta)
        self.name = 'NNGP'
        self.fatol = 1e-1 if fatol is None else fatol
        self.xatol = 1e-1 if xatol is None else xatol
        self.n = n
        self.n_restarts = kwargs.get('n_restarts', 1)
        self.nn = kwargs.get('nn', 'adaptive')
        self.seed = kwargs.get('seed', 45)
        self.rng = np.random.default_rng(self.seed)
        np.random.seed(self.seed)
        self.pool = worker_pool
        self.maxfev = 200 * len(self.theta)   # scipy default maxiter = maxfev = 200*N
        self.tot_train_t = 0
        self.train_count = 0
        self.k = 0
        self._dev_xy = None
        self._host_xy = None
        if self.nn != 'adaptive' and not 1 <= int(self.nn) <= MAX_NEIGHBOURS:
            raise ValueError(f'nn={self.nn}: the GPU nnGP correction supports 1..{MAX_NEIGHBOURS} neighbours')

    # ------------------------------------------------------------------------------ helpers
    @property
    def n_fits(self):
        return self.n * len(JITTERS) * self.n_restarts

    def n_neighbours(self):
        m = max(10, self.k + 2) if self.nn == 'adaptive' else int(self.nn)   # models.py:172-175
        if m > MAX_NEIGHBOURS:   # adaptive m = k+2 passes the bound at iteration k = 63
            raise ValueError(f"nn='adaptive' asks for m={m} neighbours at iteration {self.k}; the GPU nnGP "
                             f'correction supports up to {MAX_NEIGHBOURS}')
        return m

    def draw_thetas(self, n_predictions):
        """Initial thetas for `n_predictions` consecutive predictions (models.py:192)."""
        return self.rng.integers(-8, 0, (n_predictions * self.n_fits, len(self.theta))).astype(np.float64)

    def get_times(self):
        out = super().get_times()
        out.update({'serial_train_time': self.tot_train_t, 'calc_detail_avg': None, 'overhead': None,
                    'avg_serial_train_time': self.tot_train_t / max(self.train_count, 1)})
        return out

    def fit(self, x, y, k, *args, **kwargs):
        """models.py:157-159.  The Parareal driver hands over its device-resident training set
        (torch tensors): those are kept for the device path, and `x` / `y` stay host arrays as in
        the reference (copied from the device on first access)."""
        self.k = k
        if hasattr(x, 'data_ptr'):
            self._dev_xy = (x, y)
            self._host_xy = None
        else:
            self._dev_xy = None
            self._host_xy = (x, y)

    def _host(self):
        if self._host_xy is None:
            if self._dev_xy is None:
                raise AttributeError("'NNGP_p' has no training set yet: call fit(x, y, k) first")
            self._host_xy = tuple(v.detach().cpu().numpy() for v in self._dev_xy)
        return self._host_xy

    def _set_xy(self, i, v):
        """Reference-style assignment `mdl.x = ...` / `mdl.y = ...` (plain attributes there,
        models.py:157-159): the host pair is updated and the device copy dropped, so the next
        prediction uploads the assigned set."""
        pair = list(self._host_xy) if self._host_xy is not None else (
            [v_.detach().cpu().numpy() for v_ in self._dev_xy] if self._dev_xy is not None else [None, None])
        pair[i] = v
        self._host_xy = tuple(pair)
        self._dev_xy = None

    x = property(lambda self: self._host()[0], lambda self, v: self._set_xy(0, v))
    y = property(lambda self: self._host()[1], lambda self, v: self._set_xy(1, v))

    # ---------------------------------------------------------------------------- device path
    def predict_device(self, X, Y, rows, new_x, theta0, out=None, bias=None, preds=None,
                       fits_out=None, stream=None):
        """One correction on device tensors.  X/Y: [>=rows][n] training set, new_x: [n],
        theta0: [n_fits][2] (this prediction's draws).  Writes preds (and out = preds + bias)."""
        import torch
        m = min(self.n_neighbours(), int(rows))   # argsort(...)[:nn] on fewer rows keeps them all
        if preds is None:
            preds = torch.empty(self.n, dtype=torch.float64, device=X.device)
        jit, jp = _lib.host_doubles(JITTERS)
        st = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        _lib.check(_lib.lib().nngp_predict(
            X.data_ptr(), Y.data_ptr(), int(rows), self.n, new_x.data_ptr(), m, len(jit), jp,
            self.n_restarts, theta0.data_ptr(), float(self.fatol), float(self.xatol), self.maxfev,
            preds.data_ptr(), bias.data_ptr() if bias is not None else None,
            out.data_ptr() if out is not None else None,
            fits_out.data_ptr() if fits_out is not None else None, st))
        self.train_count += self.n_fits
        return preds

    # ------------------------------------------------------------------------- reference API
    def predict(self, new_x, prev_F=None, prev_G=None, *args, **kwargs):
        """models.py:171-183 (host arrays in/out; kNN + fits + argmin + mean on the GPU)."""
        torch = _lib.require_gpu()
        if self._dev_xy is None:   # fit() was given host arrays (or x / y were assigned)
            if self._host_xy is None or self._host_xy[0] is None or self._host_xy[1] is None:
                raise AttributeError("'NNGP_p' has no training set yet: call fit(x, y, k) first")
            self._dev_xy = (_lib.as_device(self._host_xy[0]), _lib.as_device(self._host_xy[1]))
        X, Y = self._dev_xy
        q = torch.tensor(np.asarray(new_x, dtype=np.float64).reshape(-1), device='cuda')
        th0 = torch.tensor(self.draw_thetas(1), device='cuda')
        preds = self.predict_device(X, Y, X.shape[0], q, th0)
        return preds.cpu().numpy()

    def get_preds(self, xm, ym, n, new_x, intrvl_i):
        """models.py:185-226 on already-selected neighbours: all fits, first argmin, mean."""
        torch = _lib.require_gpu()
        m = xm.shape[0]
        ins = list(product(range(n), range(len(JITTERS)), range(self.n_restarts)))
        th0 = self.draw_thetas(1)
        res = self.fit_batch(xm, ym, [i[0] for i in ins], [i[1] for i in ins], th0)
        preds = np.empty(n)
        best_th = np.empty((n, 2))
        best_j = np.empty(n, dtype=np.int32)
        per = len(JITTERS) * self.n_restarts
        for j in range(n):
            fv = res['fval'][j * per:(j + 1) * per]
            b = int(np.argmin(fv))                  # first minimum == models.py:212-215
            best_th[j] = res['theta'][j * per + b]
            best_j[j] = ins[j * per + b][1]
        preds[:] = self.gp_mean(xm, ym, new_x, best_th, best_j)
        return preds

    def fit_batch(self, xm, ym, coords, jitter_idx, theta0):
        """pool.map(_get_opt_par, ...) as one launch (nngp_nm_fit_batch)."""
        torch = _lib.require_gpu()
        xm_t = torch.tensor(np.ascontiguousarray(xm, dtype=np.float64), device='cuda')
        ym_t = torch.tensor(np.ascontiguousarray(ym, dtype=np.float64), device='cuda')
        nf = len(coords)
        c_t = torch.tensor(np.asarray(coords, dtype=np.int32), device='cuda')
        j_t = torch.tensor(np.asarray(jitter_idx, dtype=np.int32), device='cuda')
        th_t = torch.tensor(np.ascontiguousarray(theta0, dtype=np.float64), device='cuda')
        th_o = torch.empty((nf, 2), dtype=torch.float64, device='cuda')
        fv_o = torch.empty(nf, dtype=torch.float64, device='cuda')
        ne_o = torch.empty(nf, dtype=torch.int32, device='cuda')
        jit, jp = _lib.host_doubles(JITTERS)
        st = torch.cuda.current_stream().cuda_stream
        _lib.check(_lib.lib().nngp_nm_fit_batch(
            xm.shape[0], xm.shape[1], xm_t.data_ptr(), ym_t.data_ptr(), nf, c_t.data_ptr(), j_t.data_ptr(),
            len(jit), jp, th_t.data_ptr(), float(self.fatol), float(self.xatol), self.maxfev,
            th_o.data_ptr(), fv_o.data_ptr(), ne_o.data_ptr(), st))
        self.train_count += nf
        return {'theta': th_o.cpu().numpy(), 'fval': fv_o.cpu().numpy(), 'nfev': ne_o.cpu().numpy()}

    def gp_mean(self, xm, ym, new_x, theta, jitter_idx):
        torch = _lib.require_gpu()
        n = ym.shape[1]
        xm_t = torch.tensor(np.ascontiguousarray(xm, dtype=np.float64), device='cuda')
        ym_t = torch.tensor(np.ascontiguousarray(ym, dtype=np.float64), device='cuda')
        q = torch.tensor(np.asarray(new_x, dtype=np.float64).reshape(-1), device='cuda')
        th = torch.tensor(np.ascontiguousarray(theta, dtype=np.float64), device='cuda')
        ji = torch.tensor(np.asarray(jitter_idx, dtype=np.int32), device='cuda')
        out = torch.empty(n, dtype=torch.float64, device='cuda')
        jit, jp = _lib.host_doubles(JITTERS)
        _lib.check(_lib.lib().nngp_gp_mean(xm.shape[0], n, xm_t.data_ptr(), ym_t.data_ptr(), q.data_ptr(),
                                            th.data_ptr(), ji.data_ptr(), len(jit), jp, out.data_ptr(),
                                            torch.cuda.current_stream().cuda_stream))
        return out.cpu().numpy()

    @staticmethod
    def _get_opt_par(static_ins, ins, rnd):
        """models.py:228-237: one fit -> (*theta, fval, jitter, j, elapsed)."""
        st_ = time.time()
        xm, ym, fatol, xatol = static_ins
        j, jitter, _ = ins
        tmp = NNGP_p(n=ym.shape[1], N=1, fatol=fatol, xatol=xatol)
        jidx = int(np.where(JITTERS == jitter)[0][0])
        r = tmp.fit_batch(xm, ym, [j], [jidx], np.asarray(rnd, dtype=float).reshape(1, 2))
        return (*r['theta'][0], r['fval'][0], jitter, j, time.time() - st_)

    def store(self):
        """A deep copy for the result dict (models.py store): host x / y, no device tensors."""
        if self._dev_xy is not None:
            self._host()
        dev, self._dev_xy = self._dev_xy, None
        try:
            new = super().store()
        finally:
            self._dev_xy = dev
        new.pool = None
        return new

    def state_dict(self):
        st = super().state_dict()
        st['settings'] = {'theta': self.theta.tolist(), 'fatol': self.fatol, 'xatol': self.xatol,
                          'n_restarts': self.n_restarts, 'nn': self.nn, 'seed': self.seed}
        st.update({'k': self.k, 'tot_train_t': self.tot_train_t, 'train_count': self.train_count,
                   'rng': self.rng.bit_generator.state})
        return st

    def load_state(self, st):
        super().load_state(st)
        self.k, self.tot_train_t, self.train_count = st['k'], st['tot_train_t'], st['train_count']
        self.rng.bit_generator.state = st['rng']

    def restore_attrs(self, pool):
        self.pool = pool


def _select_fit(theta, fval, jitter):
    """The per-coordinate choice of models.py:388-395 / 361-365: keep fits with
    fval < 0.9 * min(fval) (all if none), then the first minimum in order (Python min, '<')."""
    fmin = np.min(fval)
    mask = fval < fmin * 0.9
    if mask.sum() == 0:
        mask[:] = True
    idx = np.nonzero(mask)[0]
    best = idx[0]
    for i in idx[1:]:
        if fval[i] < fval[best]:
            best = i
    return tuple(float(v) for v in theta[best]), float(fval[best]), float(jitter[best])


def _group_world(group):
    """(world, rank) of a torch.distributed group, (1, 0) without one."""
    import torch.distributed as dist
    if group is False or not (dist.is_available() and dist.is_initialized()):
        return 1, 0
    return dist.get_world_size(group), dist.get_rank(group)


def _gather_rows(local, group, world):
    """All-gather of equal [chunk][...] fp64 blocks in rank order over `group`: RCCL's
    all_gather_into_tensor on device tensors (an NCCL group), gloo's list form through host memory
    (several ranks sharing one GPU)."""
    import torch
    import torch.distributed as dist
    if dist.get_backend(group) == 'gloo':
        host = local.detach().cpu()
        parts = [torch.empty_like(host) for _ in range(world)]
        dist.all_gather(parts, host, group=group)
        return torch.cat(parts).to(local.device)
    out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, local.contiguous(), group=group)
    return out


class GPjax_p(ModelAbstr):
    """Full-data GParareal correction (models.py:273-473) on the GPU.

    Same constructor, attributes (thetas, jitters, hyp, fatol/xatol default 1e-4, rng =
    default_rng(45) for the random-restart fallback) and training semantics as the reference;
    the d*9 Nelder-Mead fits of a training round advance together, one batched rows x rows
    factorisation per round (nngp_gpfull_fit).  The -LML arithmetic follows the reference's
    expressions, but the Cholesky's summation order is the GPU's own (LAPACK's blocked order is
    not reproduced): parity is to tolerance and on K (tests/test_gpu_gpfull.py)."""

    def __init__(self, n, N, worker_pool=None, theta=None, jitter=None, fatol=None, xatol=None, **kwargs):
        super().__init__(N=N, **kwargs)
        if theta is None:
            theta = [1, 1]
        theta = np.array(theta)
        self.name = 'GP'
        self.hyp = np.ones((n, theta.shape[0], N))
        self.thetas = [tuple(float(v) for v in theta) for _ in range(n)]
        self.jitters = [None for _ in range(n)]
        self.fatol = 1e-4 if fatol is None else fatol
        self.xatol = 1e-4 if xatol is None else xatol
        self.theta = theta
        self.N = N
        self.n = n
        self.pool = worker_pool
        self.rng = np.random.default_rng(45)
        self.maxfev = 200 * theta.shape[0]
        self.tot_train_t = np.zeros(N)
        self.train_count = np.zeros(N)
        self.k = 0
        self.rounds = []
        # per training call: training rows and the likelihood evaluations its fits made (sum of
        # nfev = the (rows+1)^2 matrices factored), for the measured Cholesky rate (bench.py);
        # sharded over ranks, a call's entry counts every rank's fits (tot_train_t stays this rank's)
        self.call_rows, self.call_evals = [], []
        self._dev = None   # (X [rows][n], alpha [n][rows], coef [n][2]) device tensors
        # multi-GPU (the reference's pool.map over the d*9 fits, models.py:386-392):
        # the torch.distributed group the fits are sharded over by coordinate (Parareal sets it;
        # None = the default group when one is initialised, False = never shard)
        self.process_group = kwargs.get('process_group')
        self.shard_fits = kwargs.get('shard_fits', True)

    def get_times(self):
        out = super().get_times()
        with np.errstate(invalid='ignore', divide='ignore'):
            avg = (self.tot_train_t / self.train_count)[:self.k + 1]
        out.update({'serial_train_time': self.tot_train_t[:self.k + 1], 'avg_serial_train_time': avg})
        return out

    # ---------------------------------------------------------------------------- training
    def _fit_batch(self, X, Y, coords, jitters, theta0):
        """pool.map(_get_opt_par[_rnd], ...) (models.py:404-407, 355-358) as one native call."""
        import torch
        nf = len(coords)
        c = np.ascontiguousarray(coords, dtype=np.int32)
        jx, jp = _lib.host_doubles(jitters)
        t0, tp = _lib.host_doubles(np.asarray(theta0, dtype=float).reshape(nf, 2))
        th = np.empty((nf, 2))
        fv = np.empty(nf)
        ne = np.empty(nf, dtype=np.int32)
        rounds = ctypes.c_int32(0)
        ip = ctypes.POINTER(ctypes.c_int32)
        st = time.time()
        _lib.check(_lib.lib().nngp_gpfull_fit(
            X.data_ptr(), X.shape[0], self.n, Y.data_ptr(), nf, c.ctypes.data_as(ip), jp, tp, float(self.fatol),
            float(self.xatol), self.maxfev, th.ctypes.data_as(_lib._dp), fv.ctypes.data_as(_lib._dp),
            ne.ctypes.data_as(ip), ctypes.byref(rounds), torch.cuda.current_stream().cuda_stream))
        self.tot_train_t[min(self.k, self.N - 1)] += time.time() - st
        self.train_count[min(self.k, self.N - 1)] += nf
        self.rounds.append(int(rounds.value))
        self.call_rows.append(int(X.shape[0]))
        self.call_evals.append(int(ne.astype(np.int64).sum()))
        return th, fv, ne

    def _train_coord_rnd(self, X, Y, coord):
        """models.py:352-374: random restarts for a coordinate whose fits all failed."""
        tot_rnd = max(3, int(self.N / 9))
        ins = list(product([coord for _ in range(tot_rnd)], JITTERS))
        thetas = [10 ** self.rng.uniform(-4, 1, (len(self.theta))) for _ in range(len(ins))]
        th, fv, _ = self._fit_batch(X, Y, [i[0] for i in ins], [i[1] for i in ins], thetas)
        opt_params, opt_fval, opt_jitter = _select_fit(th, fv, np.array([i[1] for i in ins]))
        if np.isinf(opt_fval):
            print('random restart failed')
            opt_params, opt_fval, opt_jitter = self._train_coord_rnd(X, Y, coord)
        return opt_params, opt_fval, opt_jitter

    def _shard(self):
        """(group, world, rank, c0, c1, chunk) of the coordinate split, or None on one rank."""
        if not self.shard_fits:
            return None
        world, rank = _group_world(self.process_group)
        if world <= 1:
            return None
        chunk = (self.n + world - 1) // world
        c0, c1 = min(rank * chunk, self.n), min((rank + 1) * chunk, self.n)
        return self.process_group, world, rank, c0, c1, chunk

    def _train(self, X, Y, old_thetas):
        """models.py:376-417: every (coordinate, jitter) fit from the coordinate's old theta.
        Over several ranks each fits its own contiguous block of coordinates (every fit's
        arithmetic is independent of which others share its batch), then ONE all-gather of
        (theta, fval, nfev) gives every rank all fits; the selection, the random-restart fallback
        (whose draws come from the shared rng stream) and the weights stay replicated."""
        nj = len(JITTERS)
        sh = self._shard()
        if sh is None:
            ins = list(product(range(self.n), JITTERS))
            th, fv, _ = self._fit_batch(X, Y, [i[0] for i in ins], [i[1] for i in ins],
                                        [old_thetas[i[0]] for i in ins])
        else:
            import torch
            group, world, rank, c0, c1, chunk = sh
            buf = torch.zeros((chunk * nj, 4), dtype=torch.float64, device=X.device)
            if c1 > c0:
                ins = list(product(range(c0, c1), JITTERS))
                th_l, fv_l, ne_l = self._fit_batch(X, Y, [i[0] for i in ins], [i[1] for i in ins],
                                                   [old_thetas[i[0]] for i in ins])
                buf[:len(ins)] = torch.tensor(np.column_stack([th_l, fv_l, ne_l]), dtype=torch.float64)
            allf = _gather_rows(buf, group, world).cpu().numpy()[:self.n * nj]
            th, fv = np.ascontiguousarray(allf[:, :2]), np.ascontiguousarray(allf[:, 2])
            self.train_count[min(self.k, self.N - 1)] += self.n * nj - (c1 - c0) * nj   # all fits, as one rank counts them
            # the call's evaluations over ALL ranks' fits (the gathered nfev column), consistent
            # with train_count: bench.py's executed Cholesky rate reads these
            total = int(allf[:, 3].astype(np.int64).sum())
            if c1 > c0:
                self.call_evals[-1] = total
            else:
                self.call_rows.append(int(X.shape[0]))
                self.call_evals.append(total)
        temp = np.zeros((self.n, len(self.theta)))
        nj = len(JITTERS)
        for j in range(self.n):
            sl = slice(j * nj, (j + 1) * nj)
            opt_params, opt_fval, opt_jitter = _select_fit(th[sl], fv[sl], JITTERS)
            if np.isinf(opt_fval):
                print('------> GP trainign failed for coordinate', j)
                opt_params, opt_fval, opt_jitter = self._train_coord_rnd(X, Y, j)
            self.thetas[j] = opt_params
            self.jitters[j] = opt_jitter
            temp[j, :] = opt_params
        return temp

    def _weights(self, X, Y):
        """The posterior weights _predict memoises (models.py:441-453): alpha_j = K_j^-1 y_j for
        the chosen (theta_j, jitter_j).  The reference keys its memo by theta alone, so a
        coordinate whose theta equals an earlier coordinate's reuses that coordinate's weights
        (reproduced)."""
        import torch
        n, rows = self.n, X.shape[0]
        ip = ctypes.POINTER(ctypes.c_int32)

        def lml(c0, c1, alpha_out):
            th, tp = _lib.host_doubles(np.array(self.thetas[c0:c1], dtype=float))
            jx, jp = _lib.host_doubles(np.array(self.jitters[c0:c1], dtype=float))
            c = np.arange(c0, c1, dtype=np.int32)
            fv = np.empty(c1 - c0)
            _lib.check(_lib.lib().nngp_gpfull_lml(
                X.data_ptr(), rows, n, Y.data_ptr(), c1 - c0, c.ctypes.data_as(ip), jp, tp,
                fv.ctypes.data_as(_lib._dp), alpha_out.data_ptr(), torch.cuda.current_stream().cuda_stream))
            return fv

        sh = self._shard()
        if sh is None:
            alpha = torch.empty((n, rows), dtype=torch.float64, device=X.device)
            fv = lml(0, n, alpha)
        else:   # each rank its coordinates' weights, then one all-gather of [chunk][rows] (+ fval)
            group, world, rank, c0, c1, chunk = sh
            buf = torch.zeros((chunk, rows + 1), dtype=torch.float64, device=X.device)
            if c1 > c0:
                part = torch.empty((c1 - c0, rows), dtype=torch.float64, device=X.device)
                fv_l = lml(c0, c1, part)
                buf[:c1 - c0, 1:] = part
                buf[:c1 - c0, 0] = torch.tensor(fv_l, dtype=torch.float64)
            allb = _gather_rows(buf, group, world)[:n]
            alpha = allb[:, 1:].contiguous()
            fv = allb[:, 0].cpu().numpy()
        if np.any(np.isinf(fv)):
            raise np.linalg.LinAlgError('Matrix is not positive definite')   # np.linalg.cholesky in _predict
        first = {}
        for j in range(n):
            key = tuple(self.thetas[j])
            if key in first:
                alpha[j] = alpha[first[key]]
            else:
                first[key] = j
        coef = torch.tensor([[-0.5 * (1 / (sx * sx)), sy * sy] for sx, sy in self.thetas],
                            dtype=torch.float64, device=X.device)
        return alpha, coef

    def fit(self, x, y, k, *args, **kwargs):
        """models.py:420-425."""
        torch = _lib.require_gpu()
        self.k = k
        X, Y = _lib.as_device(x), _lib.as_device(y)
        new_hyp = self._train(X, Y, self.thetas)
        if k + 1 < self.hyp.shape[-1]:
            self.hyp[..., k + 1] = new_hyp
        self.x, self.y = x, y
        alpha, coef = self._weights(X, Y)
        self._dev = (X, alpha, coef)

    # ---------------------------------------------------------------------------- prediction
    def predict_device(self, new_x, out=None, bias=None, stream=None):
        import torch
        X, alpha, coef = self._dev
        if out is None:
            out = torch.empty(self.n, dtype=torch.float64, device=X.device)
        st = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        _lib.check(_lib.lib().nngp_gpfull_mean(
            X.data_ptr(), X.shape[0], self.n, new_x.data_ptr(), coef.data_ptr(), alpha.data_ptr(),
            bias.data_ptr() if bias is not None else None, out.data_ptr(), st))
        return out

    def predict(self, new_x, prev_F=None, prev_G=None, *args, **kwargs):
        """models.py:456-462 (host arrays in/out)."""
        torch = _lib.require_gpu()
        q = torch.tensor(np.asarray(new_x, dtype=np.float64).reshape(-1), device='cuda')
        return self.predict_device(q).cpu().numpy()

    def store(self):
        new = copy.copy(self)
        new.pool = None
        new._dev = None
        new.hyp = self.hyp[..., :self.k + 3]
        return new

    def state_dict(self):
        st = super().state_dict()
        st['settings'] = {'theta': self.theta.tolist(), 'fatol': self.fatol, 'xatol': self.xatol}
        st.update({'k': self.k, 'thetas': [list(t) for t in self.thetas], 'jitters': self.jitters,
                   'hyp': self.hyp.tolist(), 'tot_train_t': self.tot_train_t.tolist(),
                   'train_count': self.train_count.tolist(), 'rng': self.rng.bit_generator.state})
        return st

    def load_state(self, st):
        super().load_state(st)
        self.k = st['k']
        self.thetas = [tuple(t) for t in st['thetas']]
        self.jitters = list(st['jitters'])
        self.hyp = np.array(st['hyp'], dtype=float)
        self.tot_train_t = np.array(st['tot_train_t'], dtype=float)
        self.train_count = np.array(st['train_count'], dtype=float)
        self.rng.bit_generator.state = st['rng']

    def restore_attrs(self, pool):
        self.pool = pool
        self._dev = None
