"""Propagators -- the reference's SolverAbstr / SolverRK plugin surface (solver.py:21-113) with a
HIP backend.

Single-slice calls (`run_F(t0, t1, u0)`, `run_G`, their `_timed` variants) keep the reference's
signatures and numpy in/out.  The Parareal driver uses the batched device entry points
`run_F_batch` / `run_G_batch`, which integrate every slice of one iteration in ONE kernel launch
(nngp_rk_batch); that replaces `pool.map(solver.run_F_timed, ...)` at parareal.py:310-315.

Step conventions (include/nngp.h):
  step_mode='fixed'    (default)  h = (t1-t0)/steps            RK.run_get_last, RK.py:101-109
  step_mode='linspace'            h_n = t[n+1]-t[n] of np.linspace  legacy new_lib.RK, RK.py:91-99
`thresh` reproduces the paging of SolverRK._run_RK_paged (solver.py:86-99) including its quirk
(each page re-uses the full steps-1 count over 1/n_pages of the slice).
`fma=True` (opt-in; env NNGP_RK_CONTRACT=1 flips the default) runs F and G on the contracted code
object (NNGP_STEP_CONTRACT): a*b+c fused, ~25 % fewer fp64 instructions per step, end states within
1e-12 relative of the exact build instead of bitwise (tests/test_gpu_contract.py).
"""
import os
import ctypes
import time

import numpy as np

from . import _lib


def calc_time(f):
    def wrapper(*args, **kwargs):
        s_time = time.time()
        ret = f(*args, **kwargs)
        return ret, time.time() - s_time
    return wrapper


class SolverAbstr:
    """Abstract propagator: run_*(t0, t1, u0) returns the solution at t1 (solver.py:29-69)."""

    def run_F(self, t0, t1, u0):
        raise NotImplementedError('run_F not implemented')

    @calc_time
    def run_F_timed(self, t0, t1, u0):
        return self.run_F(t0, t1, u0)

    def run_F_full(self, t0, t1, u0):
        raise NotImplementedError('run_F_full not implemented')

    @calc_time
    def run_F_full_timed(self, t0, t1, u0):
        return self.run_F_full(t0, t1, u0)

    def run_G(self, t0, t1, u0):
        raise NotImplementedError('run_G not implemented')

    @calc_time
    def run_G_timed(self, t0, t1, u0):
        return self.run_G(t0, t1, u0)

    def run_G_full(self, t0, t1, u0):
        raise NotImplementedError('run_G_full not implemented')

    @calc_time
    def run_G_full_timed(self, t0, t1, u0):
        return self.run_G_full(t0, t1, u0)


def _paging_schedule(steps, thresh):
    """solver.py:91-93: the page lengths (in units of step) and the per-page step count."""
    steps = steps - 1
    n_full = int(steps / thresh)
    rem = steps % thresh
    return [thresh] * n_full + [rem] * int(rem != 0), steps


class SolverRK(SolverAbstr):
    """Fixed-step explicit RK fine (F) and coarse (G) propagators on the GPU.

    f: the VectorField returned by ODE.get_vector_field() (carries the device descriptor).
    Ng, Nf: steps per slice (modern convention, configs.py); F, G: 'RK1'|'RK2'|'RK4'|'RK8'.
    """

    def __init__(self, f, Ng, Nf, F, G, thresh=1e7, use_jax=True, step_mode='fixed', fma=None, **kwargs):
        if not hasattr(f, 'csystem'):
            raise TypeError('f must be the VectorField returned by ODE.get_vector_field()')
        self.f = f
        self.Ng = int(Ng)
        self.Nf = int(Nf)
        self.F = F
        self.G = G
        self.thresh = thresh
        if F not in _lib.TABLEAU or G not in _lib.TABLEAU:
            raise NotImplementedError('Only RK1, RK2, RK4 and RK8 are implemented')
        self.step_mode = {'fixed': _lib.STEP_FIXED, 'linspace': _lib.STEP_LINSPACE}[step_mode]
        if fma is None:
            fma = os.environ.get('NNGP_RK_CONTRACT') == '1'
        self.fma = bool(fma)
        if self.fma:
            self.step_mode |= _lib.STEP_CONTRACT

    # -------------------------------------------------------------------------------- device
    def _launch(self, method, t0, t1, steps, U0, out, stream):
        import torch
        cs = self.f.csystem(U0.device)
        st = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        _lib.check(_lib.lib().nngp_rk_batch(ctypes.byref(cs), _lib.TABLEAU[method], self.step_mode,
                                             U0.shape[0], t0.data_ptr(), t1.data_ptr(), int(steps),
                                             U0.data_ptr(), out.data_ptr(), st))
        return out

    def _run_batch(self, method, steps, t0, t1, U0, out=None, stream=None):
        """Integrate U0[i] from t0[i] to t1[i] for all i (one launch per page)."""
        import torch
        if out is None:
            out = torch.empty_like(U0)
        n = U0.shape[0]
        if n == 0:
            return out
        assert U0.dtype == torch.float64 and U0.is_contiguous() and U0.is_cuda
        if steps > self.thresh:   # paged quirk, solver.py:86-99 -- rare; host-side schedule
            t0h = t0.detach().cpu().numpy() if torch.is_tensor(t0) else np.asarray(t0, dtype=float)
            t1h = t1.detach().cpu().numpy() if torch.is_tensor(t1) else np.asarray(t1, dtype=float)
            iters, psteps = _paging_schedule(steps, self.thresh)
            step = (t1h - t0h) / psteps
            cur = U0
            a = t0h.copy()
            for temp_steps in iters:
                b = a + step * temp_steps
                ta = torch.tensor(a, dtype=torch.float64, device=U0.device)
                tb = torch.tensor(b, dtype=torch.float64, device=U0.device)
                self._launch(method, ta, tb, psteps, cur, out, stream)
                cur = out
                a = b
            return out
        if not torch.is_tensor(t0):
            t0 = torch.tensor(np.asarray(t0, dtype=float), device=U0.device)
            t1 = torch.tensor(np.asarray(t1, dtype=float), device=U0.device)
        return self._launch(method, t0, t1, steps, U0, out, stream)

    def coarse_is_paged(self):
        return self.Ng > self.thresh

    def initial_coarse(self, t_dev, UG, N):
        """Initial coarse sweep (parareal.py:265-270): UG[i+1] = G(t[i], t[i+1], UG[i]), one
        slice after the other."""
        for i in range(N):
            self.run_G_batch(t_dev[i:i + 1], t_dev[i + 1:i + 2], UG[i:i + 1], out=UG[i + 1:i + 2])

    def run_F_batch(self, t0, t1, U0, out=None, stream=None):
        return self._run_batch(self.F, self.Nf, t0, t1, U0, out, stream)

    def run_G_batch(self, t0, t1, U0, out=None, stream=None):
        return self._run_batch(self.G, self.Ng, t0, t1, U0, out, stream)

    # -------------------------------------------------------------------------- reference API
    def _single(self, method, steps, t0, t1, u0):
        torch = _lib.require_gpu()
        U0 = torch.tensor(np.asarray(u0, dtype=np.float64).reshape(1, -1), device='cuda')
        out = self._run_batch(method, steps, np.array([t0], dtype=float), np.array([t1], dtype=float), U0)
        return out[0].cpu().numpy()

    def run_F(self, t0, t1, u0):
        return self._single(self.F, self.Nf, t0, t1, u0)

    def run_G(self, t0, t1, u0):
        return self._single(self.G, self.Ng, t0, t1, u0)

    def _full(self, method, steps, t0, t1, u0):
        """Whole trajectory on the np.linspace grid (RK.run, RK.py:91-99): one launch per point."""
        torch = _lib.require_gpu()
        steps = int(steps)
        t = np.linspace(t0, t1, num=steps + 1)
        out = np.empty((steps + 1, len(u0)))
        out[0] = u0
        cur = torch.tensor(np.asarray(u0, dtype=np.float64).reshape(1, -1), device='cuda')
        nxt = torch.empty_like(cur)
        mode = self.step_mode
        self.step_mode = _lib.STEP_FIXED | (mode & _lib.STEP_CONTRACT)
        try:
            for n in range(steps):
                ta = torch.tensor([t[n]], dtype=torch.float64, device='cuda')
                tb = torch.tensor([t[n + 1]], dtype=torch.float64, device='cuda')
                self._launch(method, ta, tb, 1, cur, nxt, None)
                cur, nxt = nxt, cur
                out[n + 1] = cur[0].cpu().numpy()
        finally:
            self.step_mode = mode
        return out

    def run_F_full(self, t0, t1, u0):
        return self._full(self.F, self.Nf, t0, t1, u0)

    def run_G_full(self, t0, t1, u0):
        return self._full(self.G, self.Ng, t0, t1, u0)
