"""CPU: the C-ABI library loads, exports every entry point include/nngp.h declares, and validates
arguments (error codes + thread-local message) before touching the GPU."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, 'include', 'nngp.h')).read()
    return sorted(set(re.findall(r'^\s*(?:const\s+)?\w+\s*\*?\s*(nngp_\w+)\s*\(', src, re.M)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ['nngp_rk_batch', 'nngp_rk_batch_grid', 'nngp_rhs_batch', 'nngp_parareal_update',
              'nngp_knn', 'nngp_nm_fit_batch', 'nngp_gp_mean', 'nngp_predict', 'nngp_last_error']:
        assert s in syms


def test_library_exports_every_declared_symbol():
    import nngp_amd
    L = nngp_amd.lib()
    for s in declared_symbols():
        assert hasattr(L, s), s
    assert sorted(nngp_amd._lib.EXPORTS) == declared_symbols()
    assert L.nngp_abi_version() == 1
    assert L.nngp_device_count() >= 0


def test_argument_errors_are_reported_without_a_gpu():
    import nngp_amd
    L = nngp_amd.lib()
    assert L.nngp_rk_batch(None, 4, 0, 1, None, None, 10, None, None, None) == -1
    assert b'sys is NULL' in L.nngp_last_error()
    cs = nngp_amd._lib.CSystem(0, 3, 0, 0, (ctypes.c_double * 4)(), None)
    assert L.nngp_rk_batch(ctypes.byref(cs), 4, 0, 1, None, None, 0, None, None, None) == -1
    assert b'steps' in L.nngp_last_error()
    assert L.nngp_predict(None, None, 10, 3, None, 5, 9, None, 1, None, 0.1, 0.1, 400, None, None, None,
                          None, None) == -1
    assert L.nngp_nm_fit_batch(65, 3, None, None, 1, None, None, 9, None, None, 0.1, 0.1, 400, None, None,
                               None, None) == -1
    assert b"m <= 64" in L.nngp_last_error()
    assert L.nngp_rk_batch(ctypes.byref(cs), 4, 0, 0, None, None, 10, None, None, None) == 0   # empty batch


def test_product_path_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    import nngp_amd
    ode = nngp_amd.Lorenz(normalization='-11')
    s = nngp_amd.SolverRK(ode.get_vector_field(), Ng=6, Nf=45, F='RK4', G='RK4')
    with pytest.raises(nngp_amd.NNGPError):
        s.run_F(0.0, 0.5, ode.get_init_cond())
    p = nngp_amd.Parareal(ode, s, [0, 18], 4)
    with pytest.raises(nngp_amd.NNGPError):
        p.run(model='nngp', nn=10)
