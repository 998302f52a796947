"""Pairs (oracle System, product ODE factory) for every fixture key in tests/golden/rhs.npz and rk.npz."""
import oracle as O


def oracle_system(key):
    return {
        'lorenz': lambda: O.System('lorenz'),
        'hopf': lambda: O.System('hopf', param=(500.0,)),
        'tomlab': lambda: O.System('tomlab'),
        'fhn_ode': lambda: O.System('fhn_ode'),
        'rossler': lambda: O.System('rossler'),
        'brus': lambda: O.System('brus'),
        'dblpend': lambda: O.System('dblpend'),
        'lorenz_id': lambda: O.System('lorenz', normalized=False),
        'burgers128': lambda: O.System('burgers', d=128, param=(0.01,), mn=0, mx=1),
        'burgers16': lambda: O.System('burgers', d=16, param=(0.01,), mn=0, mx=1),
        'fhnpde10': lambda: O.System('fhn_pde', nx=10, normalized=False),
        'fhnpde10_n': lambda: O.System('fhn_pde', nx=10, mn=-1, mx=1),
        'fhnpde4': lambda: O.System('fhn_pde', nx=4, normalized=False),
    }[key]()


def product_ode(g, key):
    return {
        'lorenz': lambda: g.Lorenz(normalization='-11'),
        'hopf': lambda: g.Hopf(normalization='-11'),
        'tomlab': lambda: g.ThomasLabyrinth(normalization='-11'),
        'fhn_ode': lambda: g.FHN_ODE(normalization='-11'),
        'rossler': lambda: g.Rossler(normalization='-11'),
        'brus': lambda: g.Brusselator(normalization='-11'),
        'dblpend': lambda: g.DblPend(normalization='-11'),
        'lorenz_id': lambda: g.Lorenz(),
        'burgers128': lambda: g.Burgers(d_x=128, normalization='-11'),
        'burgers16': lambda: g.Burgers(d_x=16, normalization='-11'),
        'fhnpde10': lambda: g.FHN_PDE(d_x=10),
        'fhnpde10_n': lambda: g.FHN_PDE(d_x=10, normalization='-11'),
        'fhnpde4': lambda: g.FHN_PDE(d_x=4),
    }[key]()


KEYS = ['lorenz', 'hopf', 'tomlab', 'fhn_ode', 'rossler', 'brus', 'dblpend', 'lorenz_id', 'burgers128',
        'burgers16', 'fhnpde10', 'fhnpde10_n', 'fhnpde4']
RK_KEYS = [k for k in KEYS if k != 'lorenz_id']
# ODEs whose RHS restatement is bit-exact vs the reference (PDEs sum dense-row products in
# BLAS order; FHN_ODE's u**3 is x*(x*x) per jax while the numpy stand-in used pow; the
# trigonometric fields use the repo's fully specified sin/cos, ~1 ulp from the reference's libm,
# and are bit-exact GPU vs oracle instead)
EXACT = {'lorenz', 'hopf', 'rossler', 'brus', 'lorenz_id'}
TRIG = {'tomlab', 'dblpend'}
