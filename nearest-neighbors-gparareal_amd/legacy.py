"""The legacy monolith's surface (new_lib.py) -- the API every published scalability run used
(Burgers.py, Hopf.py, TomLab.py, FHN_PDE.py).

Differences from the modern API (parareal.py/solver.py), all reproduced here:
  * Ng, Nf are TOTAL step counts over tspan (new_lib.py:849-855, must divide: Ng % N == Nf % Ng == 0);
  * a slice is integrated on np.linspace(t_i, t_{i+1}, int(Nf/N)+1) -- h_n = t[n+1]-t[n], not a
    fixed dt (RK_last -> RK, new_lib.py:57-69, 87-108);
  * RK_last's paging quirk: when the point count exceeds RK_thresh, every page re-uses the full
    per-slice point count over a 1/n_pages sub-interval (new_lib.py:59-66; float page lengths
    allowed, e.g. TomLab's remainder sliver);
  * the initial coarse solution is ONE coarse integration over the whole span, sub-sampled at the
    slice boundaries (new_lib.py:902-906) -> nngp_rk_batch_grid;
  * run(..., lag_k=...) trains the model on the last lag_k iterations only (new_lib.py:980-987).
The model and the Parareal loop are shared with the modern driver.  `f` must be a VectorField of
this package (ODE.get_vector_field()): the right-hand sides run inside the HIP propagator.
"""
import ctypes

import numpy as np

from . import _lib
from .parareal import Parareal as _Parareal
from .solver import SolverRK
from .systems import FHN_ODE, DblPend, Hopf, Lorenz, Rossler


def _legacy_pages(t_steps, thresh):
    """RK_last's schedule (new_lib.py:59-66): (page lengths in units of `step`, points per page)
    when paged, else None."""
    if t_steps > thresh:
        t_steps = t_steps - 1
        iters = [thresh] * int(t_steps / thresh) + [t_steps % thresh] * (t_steps % thresh != 0)
        return iters, t_steps
    return None


class LegacySolverRK(SolverRK):
    """new_lib's propagators on the GPU: RK_last / RK_last_t / RK_t (new_lib.py:57-85)."""

    def __init__(self, f, N, Ng, Nf, F, G, RK_thresh=1e7):
        if (Ng % N != 0) or (Nf % Ng != 0):
            raise Exception('Nf must be a multiple of Ng and Ng must be a multiple of N - change time steps!')
        super().__init__(f, Ng=Ng // N, Nf=Nf // N, F=F, G=G, thresh=float('inf'), step_mode='linspace')
        self.N, self.Ng_total, self.Nf_total = int(N), int(Ng), int(Nf)
        self.RK_thresh = RK_thresh

    def _rk_last(self, method, per_slice, t0, t1, U0, out, stream):
        import torch
        if out is None:
            out = torch.empty_like(U0)
        if U0.shape[0] == 0:
            return out
        t_steps = int(per_slice) + 1                 # int(Nf/N)+1 points (new_lib.py:940, 997)
        pages = _legacy_pages(t_steps, self.RK_thresh)
        if pages is None:
            return self._launch(method, t0, t1, t_steps - 1, U0, out, stream)
        iters, pts = pages
        t_s = t0.detach().cpu().numpy() if torch.is_tensor(t0) else np.asarray(t0, dtype=float)
        t_e = t1.detach().cpu().numpy() if torch.is_tensor(t1) else np.asarray(t1, dtype=float)
        step = (t_e - t_s) / pts
        cur = U0
        for temp in iters:                           # each page: linspace(t_s, t_end, num=pts)
            t_end = t_s + step * temp
            self._launch(method, torch.tensor(t_s, dtype=torch.float64, device=U0.device),
                         torch.tensor(t_end, dtype=torch.float64, device=U0.device), pts - 1, cur, out, stream)
            cur = out
            t_s = t_end
        return out

    def run_F_batch(self, t0, t1, U0, out=None, stream=None):
        return self._rk_last(self.F, self.Nf, t0, t1, U0, out, stream)

    def run_G_batch(self, t0, t1, U0, out=None, stream=None):
        return self._rk_last(self.G, self.Ng, t0, t1, U0, out, stream)

    def coarse_is_paged(self):
        return _legacy_pages(self.Ng + 1, self.RK_thresh) is not None

    def initial_coarse(self, t_dev, UG, N):
        """RK(np.linspace(t[0], t[-1], Ng+1)) sub-sampled every Ng/N points (new_lib.py:902-906):
        slice i continues the SAME global grid for grid steps i*Ng/N .. (i+1)*Ng/N - 1."""
        import torch
        cs = self.f.csystem(UG.device)
        st = torch.cuda.current_stream().cuda_stream
        per = self.Ng
        j0 = torch.arange(N, dtype=torch.int64, device=UG.device) * per
        for i in range(N):
            _lib.check(_lib.lib().nngp_rk_batch_grid(
                ctypes.byref(cs), _lib.TABLEAU[self.G], 1, t_dev[0:1].data_ptr(), t_dev[N:N + 1].data_ptr(),
                self.Ng_total, j0[i:i + 1].data_ptr(), per, UG[i:i + 1].data_ptr(), UG[i + 1:i + 2].data_ptr(), st))


class Parareal(_Parareal):
    """new_lib.Parareal(f, tspan, u0, N, Ng, Nf, epsilon, F, G, ode_name) (new_lib.py:790-841).
    `RK_thresh` may be (re)assigned before run(), as the scalability scripts do."""

    def __init__(self, f=None, tspan=None, u0=None, N=None, Ng=None, Nf=None, epsilon=None, F=None, G=None,
                 ode_name='No-Name', normalization='-11', RK_thresh=1e7, verbose='v', process_group=None, **kwargs):
        if any(v is None for v in (f, tspan, u0, N, Ng, Nf, epsilon, F, G)):   # new_lib.py:643-646
            f, tspan, u0, epsilon, N, Ng, Nf, G, F, self.data_tr, self.data_tr_inv = Systems(
                ode_name, normalization=normalization, u0=u0, epsilon=epsilon).fetch()
        else:
            self.data_tr = self.data_tr_inv = lambda x: x
        if not hasattr(f, 'csystem'):
            raise TypeError('f must be the VectorField of an nngp_amd ODE (ode.get_vector_field())')
        self.RK_thresh = RK_thresh
        self.Ng, self.Nf, self.F, self.G = int(Ng), int(Nf), F, G
        solver = LegacySolverRK(f, N, Ng, Nf, F, G, RK_thresh)
        super().__init__(f.ode, solver, tspan, N, epsilon=epsilon, verbose=verbose, process_group=process_group)
        self.f = f
        self.u0 = np.asarray(u0, dtype=float)
        self.ode_name = ode_name
        self.n = self.u0.shape[0]

    def _setup_solver(self):
        s, N = self.solver, self.N
        Ng, Nf = int(self.Ng), int(self.Nf)
        if (Ng % N != 0) or (Nf % Ng != 0):
            raise Exception('Nf must be a multiple of Ng and Ng must be a multiple of N - change time steps!')
        if self.F not in _lib.TABLEAU or self.G not in _lib.TABLEAU:
            raise NotImplementedError('Only RK1, RK2, RK4 and RK8 are implemented')
        s.Ng, s.Nf, s.Ng_total, s.Nf_total = Ng // N, Nf // N, Ng, Nf
        s.F, s.G = self.F, self.G
        s.RK_thresh = self.RK_thresh

    def load_int_dump(self, *args, **kwargs):
        self._setup_solver()
        return super().load_int_dump(*args, **kwargs)

    def run(self, *args, **kwargs):
        # new_lib's _parareal reads self.Ng / self.Nf / self.F / self.G / self.RK_thresh when it
        # runs (new_lib.py:902-997), and the scalability scripts re-assign them after construction
        # (Hopf.py:68-69: s.Nf = s.Nf * 10000; s.RK_thresh = s.Nf/s.N/scaling)
        self._setup_solver()
        return super().run(*args, **kwargs)


class Systems:
    """new_lib.Systems name registry (new_lib.py:1451-1758): 'rossler_long', 'non_aut{N}', 'fhn',
    'dbl_pend', 'lorenz', with a trailing '_n' selecting the '-11' normalisation.  fetch() returns
    (f, tspan, u0, epsilon, N, Ng, Nf, G, F, data_tr, data_tr_inv) like the reference."""
    avail_odes = ['rossler_long', 'non_aut', 'fhn', 'dbl_pend', 'brus_2d', 'lorenz']

    def __init__(self, ode_name, normalization='-11', **kwargs):
        if sum(map(lambda x: x in ode_name.lower(), self.avail_odes)) != 1:
            raise Exception(f'Unknown ode {ode_name}')
        if normalization not in ['-11', 'identity']:
            raise Exception('Unknown value of normalizaiton')
        if ode_name.lower()[-2:] == '_n':
            self.normalization, self.normalize = normalization, True
            ode_name = ode_name[:-2]
        else:
            self.normalization, self.normalize = 'identity', False
        self.name = ode_name.lower()
        self.kwargs = dict(kwargs)
        if 'non_aut' in self.name:
            try:
                self.kwargs['N'] = int(ode_name[7:])
            except ValueError:
                raise Exception(f'Invalid interval number for non aut system: {ode_name}, {ode_name[7:]}') from None
        if self.name == 'brus_2d':
            raise NotImplementedError('brus_2d (2-D Brusselator PDE) is outside the BASELINE configs')

    def _cfg(self):
        kw = self.kwargs
        eps = kw.get('epsilon') if kw.get('epsilon') is not None else 10 ** (-6)
        norm = '-11' if self.normalize and self.normalization == '-11' else None
        if self.name == 'fhn':                          # get_fhn, new_lib.py:1547-1566
            N = 40
            Ng = N * 4
            return FHN_ODE(normalization=norm), [0, 40], eps, N, Ng, int(160000 / 160 * Ng), 'RK2', 'RK4'
        if self.name == 'rossler_long':                 # get_rossler_long: doubled span
            return Rossler(normalization=norm), [0, 340], eps, 40, 90000, 4500000, 'RK1', 'RK4'
        if 'non_aut' in self.name:                      # get_non_aut
            return Hopf(normalization=norm), [-20, 500], eps, kw['N'], 2 * 1024, 2 * 1024 * 85, 'RK1', 'RK8'
        if self.name == 'dbl_pend':
            N = 32
            Ng = 3072 + N
            return DblPend(normalization=norm), [0, 80], eps, N, Ng, Ng * 70, 'RK1', 'RK8'
        if self.name == 'lorenz':                       # get_lorenz (default epsilon 1e-8)
            N = 50
            Ng = N * 6
            eps = kw.get('epsilon') if kw.get('epsilon') is not None else 10 ** (-8)
            return Lorenz(normalization=norm), [0, 18], eps, N, Ng, Ng * 75, 'RK4', 'RK4'
        raise Exception(f'Unknown ode {self.name}')

    def fetch(self):
        ode, tspan, eps, N, Ng, Nf, G, F = self._cfg()
        u0 = ode.get_init_cond() if self.kwargs.get('u0') is None else ode.normalizer.fit(self.kwargs['u0'])
        nz = ode.normalizer
        return (ode.get_vector_field(), tspan, u0, eps, N, Ng, Nf, G, F, nz.fit, nz.inverse)
