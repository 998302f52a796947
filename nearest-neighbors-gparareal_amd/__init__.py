"""nnGParareal on MI355X: the reference's Parareal / SolverRK / NNGP_p plugin surface with the
fine RK propagator and the nearest-neighbour GP correction as hand-written HIP kernels for gfx950
(csrc/, C-ABI in include/nngp.h).  Import as `nngp_amd` (see nngp_amd.py at the repo root)."""
from . import _lib, legacy
from ._lib import NNGPError, build, lib
from .configs import Config
from .models import BareParareal, GPjax_p, ModelAbstr, NNGP_p
from .parareal import GpuPool, MyPool, Parareal, PararealLight
from .solver import SolverAbstr, SolverRK
from .systems import (ODE, Brusselator, Burgers, DblPend, FHN_ODE, FHN_PDE, Hopf, Lorenz, Rossler,
                      ThomasLabyrinth, VectorField)
from .utils import Normalize

__all__ = ['Config', 'BareParareal', 'ModelAbstr', 'NNGP_p', 'GpuPool', 'MyPool', 'Parareal',
           'SolverAbstr', 'SolverRK', 'ODE', 'Brusselator', 'Burgers', 'DblPend', 'FHN_ODE',
           'FHN_PDE', 'Hopf', 'Lorenz', 'Rossler', 'ThomasLabyrinth', 'VectorField', 'Normalize',
           'NNGPError', 'build', 'lib']
