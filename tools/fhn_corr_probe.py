"""GPU probe: the FHN-PDE d = 800 nnGP correction (m = 20, R = 1: 7 200 fits) and an 8-GPU rank's
coordinate share (100 coordinates, 900 fits) on bench.py's synthetic 3 000-row training set --
bench.py fhn_pde_strong's correction_ms / correction_ms_100_coords -- alternating an environment
knob between two values.

    python tools/fhn_corr_probe.py [KNOB V_A V_B] [n_pred]"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nngp_amd as g  # noqa: E402
from nngp_amd.models import JITTERS  # noqa: E402


def main():
    knob, va, vb = (sys.argv[1:4] if len(sys.argv) > 3 else ('NNGP_NM_LEVEL2', '1', '2'))
    n_pred = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    torch.cuda.set_device(0)
    d, rows, m = 800, 3000, 20
    rng = np.random.default_rng(0)
    X = np.clip(np.cumsum(0.01 * rng.standard_normal((rows, d)), axis=0), -1, 1)
    Y = 0.02 * np.sin(2 * X)
    dev = lambda a: torch.tensor(a, dtype=torch.float64, device='cuda')
    mdl = g.NNGP_p(n=d, N=4, nn=m, n_restarts=1, seed=45)
    th0 = dev(mdl.draw_thetas(1))
    Xd, Yd = dev(X), dev(Y)
    jit = np.ascontiguousarray(JITTERS)
    jp = jit.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    lib = g.lib()
    qs = [Xd[(97 * j) % rows] + 1e-3 for j in range(n_pred)]
    st = torch.cuda.current_stream().cuda_stream

    def run(c1, out):
        for q in qs:
            g._lib.check(lib.nngp_predict_range(Xd.data_ptr(), Yd.data_ptr(), rows, d, q.data_ptr(), m, len(jit), jp,
                                                1, th0.data_ptr(), 0, c1, 0.1, 0.1, 400, out.data_ptr(), st))

    ref = {}
    for c1 in (d, 100):
        out = torch.empty(c1, dtype=torch.float64, device='cuda')
        for v in (va, vb, va, vb):
            os.environ[knob] = v
            run(c1, out)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(c1, out)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / n_pred
            bits = out.cpu().numpy().tobytes()
            same = ref.setdefault(c1, bits) == bits
            print(f'{c1} coordinates {knob}={v}: {ms:.3f} ms per correction; bitwise the first: {same}', flush=True)


if __name__ == '__main__':
    main()
