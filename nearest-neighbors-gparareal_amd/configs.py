"""Per-system Parareal configurations -- restates the reference's configs.Config
(configs.py:6-185): tspan, N, per-slice coarse/fine step counts Ng/N and Nf/N, tableaux."""
import numpy as np

from .systems import FHN_ODE, FHN_PDE, Rossler, Hopf, DblPend, Brusselator, Lorenz, ThomasLabyrinth, ODE


class Config:
    def _fhn_ode(self, *args, **kwargs):
        tspan, N = [0, 40], 40
        Ng = N * 4
        Nf = int(160000 / 160 * Ng)
        return {'tspan': tspan, 'u0': np.array([-1, 1]), 'N': N, 'Ng': Ng / N, 'Nf': Nf / N,
                'G': 'RK2', 'F': 'RK4'}

    def _rossler(self, *args, **kwargs):
        N, Ng, Nf = 20, 45000, 2250000
        return {'tspan': [0, 170 * 2], 'u0': np.array([0, -6.78, 0.02]), 'N': N * 2,
                'Ng': Ng * 2 / (N * 2), 'Nf': Nf * 2 / (N * 2), 'G': 'RK1', 'F': 'RK4'}

    def _hopf(self, N, *args, **kwargs):
        if N is None:
            raise Exception('N must be provided')
        Ng = 2 * 1024
        Nf = Ng * 85
        return {'tspan': [-20, 500], 'u0': np.array([0.1, 0.1, -20]), 'N': N, 'Ng': Ng / N, 'Nf': Nf / N,
                'G': 'RK1', 'F': 'RK8'}

    def _pend(self, *args, **kwargs):
        N = 32
        Ng = 3072 + N
        Nf = Ng * 70
        return {'tspan': [0, 80], 'u0': np.array([-0.5, 0, 0, 0]), 'N': N, 'Ng': Ng / N, 'Nf': Nf / N,
                'G': 'RK1', 'F': 'RK8'}

    def _brus(self, *args, **kwargs):
        N = 25
        Ng = N * 10
        Nf = Ng * 100
        return {'tspan': [0, 100], 'u0': np.array([1, 3.07]), 'N': N, 'Ng': Ng / N, 'Nf': Nf / N,
                'G': 'RK4', 'F': 'RK4'}

    def _lorenz(self, *args, **kwargs):
        N = 50
        Ng = N * 6
        Nf = Ng * 75
        return {'tspan': [0, 18], 'u0': np.array([-15, -15, 20]), 'N': N, 'Ng': Ng / N, 'Nf': Nf / N,
                'G': 'RK4', 'F': 'RK4'}

    def _tomlab(self, N, *args, **kwargs):
        tot = {32: 10, 64: 10, 128: 40, 256: 100, 512: 100}
        if N not in tot:
            raise Exception('Invalid N value')
        Ng = N * 10
        Nf = Ng * int(np.ceil(1e6 / Ng))
        return {'tspan': [0, tot[N]], 'u0': np.array([4.6722764, 5.2437205e-10, -6.4444208e-10]), 'N': N,
                'Ng': Ng / N, 'Nf': Nf / N, 'G': 'RK1', 'F': 'RK4'}

    def fhn_pde(self, dx, *args, **kwargs):
        N = 512
        table = {10: (3, 150, 'RK2'), 12: (12, 550, 'RK2'), 14: (25, 950, 'RK2'), 16: (25, 1100, 'RK4')}
        mul, T, G = table.get(dx, (25, 1100, 'RK4'))
        Ng = N * mul
        Nf = int(np.ceil(1e4 / Ng) * Ng)
        return {'tspan': [0, T], 'N': N, 'Ng': Ng / N, 'Nf': Nf / N, 'G': G, 'F': 'RK8'}

    def __init__(self, ode: ODE, N=None, d_x=None):
        if isinstance(ode, FHN_ODE):
            config = self._fhn_ode()
        elif isinstance(ode, Rossler):
            config = self._rossler()
        elif isinstance(ode, Hopf):
            config = self._hopf(N)
            ode.name += f'_{N}'
        elif isinstance(ode, DblPend):
            config = self._pend()
        elif isinstance(ode, Brusselator):
            config = self._brus()
        elif isinstance(ode, Lorenz):
            config = self._lorenz()
        elif isinstance(ode, ThomasLabyrinth):
            config = self._tomlab(N)
            ode.name += f'_{N}'
        elif isinstance(ode, FHN_PDE):
            config = self.fhn_pde(d_x)
        else:
            raise Exception('No config for input ODE')
        if 'u0' in config:
            ode.set_default_init_cond(config['u0'])
        self.config = config

    def _enforce_types(self, config):
        for key, val in config.items():
            if key in ['N', 'Ng', 'Nf']:
                config[key] = int(val)
            elif key in ['u0']:
                config[key] = np.array(val)
        return config

    def get(self):
        return self._enforce_types(self.config)
