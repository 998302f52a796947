"""ODE / PDE systems -- same classes, constructor arguments, bounds and initial conditions as the
reference's systems.py (modern API).  The right-hand side itself is evaluated on the GPU inside
the HIP propagator (csrc/nngp_rk.hip); `get_vector_field()` returns a `VectorField` that
carries the device descriptor (struct nngp_system) and, when called as f(t, u), evaluates the
RHS on the GPU through nngp_rhs_batch.

Reference: /root/reference/systems.py (ODE 23-77, FHN_ODE 80-106, Rossler 109-137, Hopf 140-172,
DblPend 175-199, Brusselator 202-222, Lorenz 225-247, ThomasLabyrinth 250-288, FHN_PDE 291-398,
Burgers 402-459).  DiffReact (463-577) is not in the BASELINE configs and is not built.
"""
import ctypes

import numpy as np

from . import _lib
from .utils import Normalize


class VectorField:
    """Device-side vector field f_n(t, u) = f(inverse(u)) * scale (systems.py:32-44)."""

    def __init__(self, ode):
        self.ode = ode
        self._dev = {}

    def csystem(self, device):
        """struct nngp_system for `device` (norm table uploaded once and kept alive)."""
        import torch
        key = str(device)
        if key not in self._dev:
            ode = self.ode
            table = ode.normalizer.device_table(ode.d) if ode.normalized else None
            norm_t = None
            if table is not None:
                norm_t = torch.tensor(table, dtype=torch.float64, device=device)
            p = (ctypes.c_double * 4)(*(list(ode.param) + [0.0] * (4 - len(ode.param))))
            cs = _lib.CSystem(ode.kind, ode.d, ode.nx, int(ode.normalized), p,
                              norm_t.data_ptr() if norm_t is not None else None)
            cs._keep_alive = norm_t   # the struct holds a raw device pointer into this tensor
            self._dev[key] = (cs, norm_t)
        return self._dev[key][0]

    def __call__(self, t, u):
        torch = _lib.require_gpu()
        u = np.asarray(u, dtype=np.float64)
        single = u.ndim == 1
        U = torch.tensor(np.atleast_2d(u), dtype=torch.float64, device='cuda')
        out = torch.empty_like(U)
        st = torch.cuda.current_stream().cuda_stream
        _lib.check(_lib.lib().nngp_rhs_batch(ctypes.byref(self.csystem(U.device)), U.shape[0],
                                              U.data_ptr(), out.data_ptr(), st))
        r = out.cpu().numpy()
        return r[0] if single else r


class ODE():
    kind = None
    nx = 0

    def __init__(self, name, mn, mx, u0, normalization=None, use_jax=True, param=()):
        self.name = name
        self.normalizer = Normalize(mn, mx, normalization)
        self.normalized = self.normalizer.norm_type == '-11'
        self.u0 = self.normalizer.fit(u0)
        self.use_jax = use_jax       # accepted for signature compatibility; unused
        self.d = int(np.asarray(u0).shape[0])
        self.param = tuple(param)

    def get_vector_field(self):
        return VectorField(self)

    def set_default_init_cond(self, u0):
        self.u0 = self.normalizer.fit(u0)

    def get_init_cond(self, *args, u0=None, **kwargs):
        if u0 is None:
            u0 = self.u0
        else:
            u0 = self.normalizer.fit(u0)
        return np.array(u0, dtype=float)

    def get_dim(self):
        return self.u0.shape[0]


class FHN_ODE(ODE):
    kind = _lib.SYS_FHN_ODE

    def __init__(self, **kwargs):
        mn, mx = np.array([[-2, -1], [2.1, 1.2]])
        super().__init__('FHN_ODE', mn, mx, np.array([-1, 1]), **kwargs)


class Rossler(ODE):
    kind = _lib.SYS_ROSSLER

    def __init__(self, **kwargs):
        mn, mx = np.array([[-10, -11, 0], [12, 8, 23]])
        super().__init__('Rossler', mn, mx, np.array([0, -6.78, 0.02]), **kwargs)


class Hopf(ODE):
    kind = _lib.SYS_HOPF

    def __init__(self, tspan=[-20, 500], **kwargs):
        mn, mx = np.array([[-23, -23, 0], [23, 23, 1]])
        u0 = np.array([0.1, 0.1, tspan[0]])
        self.maxtime = tspan[1]
        super().__init__('Hopf', mn, mx, u0, param=(float(tspan[1]),), **kwargs)


class DblPend(ODE):
    kind = _lib.SYS_DBL_PEND

    def __init__(self, **kwargs):
        mn, mx = np.array([[-2, -2.5, -17, -3.5], [2, 2.5, 1, 3.5]])
        super().__init__('DblPend', mn, mx, np.array([-0.5, 0, 0, 0]), **kwargs)


class Brusselator(ODE):
    kind = _lib.SYS_BRUSSELATOR

    def __init__(self, **kwargs):
        mn, mx = np.array([[0.4, 0.9], [4, 5]])
        super().__init__('Brusselator', mn, mx, np.array([1, 3.07]), **kwargs)


class Lorenz(ODE):
    kind = _lib.SYS_LORENZ

    def __init__(self, **kwargs):
        mn, mx = np.array([[-17.1, -23, 6], [18.1, 25, 45]])
        super().__init__('Lorenz', mn, mx, np.array([-15, -15, 20]), **kwargs)


class ThomasLabyrinth(ODE):
    kind = _lib.SYS_THOMAS_LABYRINTH

    def __init__(self, **kwargs):
        mn, mx = np.array([[-12, -12, -12], [12, 12, 12]])
        u0 = np.array([4.6722764, 5.2437205e-10, -6.4444208e-10])
        super().__init__('ThomasLabyrinth', mn, mx, u0, **kwargs)


class FHN_PDE(ODE):
    """2-D FitzHugh-Nagumo on a d_x x d_x periodic grid, d = 2 d_x^2 (systems.py:291-398).
    u0 reproduces the reference's seeded draw (systems.py:303-312: np.random.seed(seed), then a
    Generator over the legacy global bit generator)."""
    kind = _lib.SYS_FHN_PDE

    def __init__(self, d_x, seed=45, **kwargs):
        self.d_x = self.d_y = d_x
        d = 2 * (d_x * d_x)
        self.nx = d_x
        mn, mx = np.array([[-1] * d, [1] * d])
        np.random.seed(seed)
        if hasattr(np.random, 'get_bit_generator'):
            rng = np.random.Generator(np.random.get_bit_generator())
        else:
            rng = np.random.default_rng(seed)
        u0 = rng.uniform(size=d)
        super().__init__(f'FHN_PDE_{d_x}', mn, mx, u0, **kwargs)


class Burgers(ODE):
    """Viscous Burgers on d_x periodic points (systems.py:402-459); nu = param[0]."""
    kind = _lib.SYS_BURGERS

    def __init__(self, d_x, nu=1 / 100, **kwargs):
        self.d_x = d_x
        self.nu = nu
        self.nx = d_x
        mn, mx = np.array([[0] * d_x, [1] * d_x])
        x_fine = np.linspace(-1, 1, num=(d_x - 1) + 1)
        u0 = 0.5 * (np.cos(4.5 * np.pi * x_fine) + 1)
        super().__init__(f'Burgers_{d_x}', mn, mx, u0, param=(float(nu),), **kwargs)
