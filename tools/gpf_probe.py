"""GPU probe: one batched full-GP -LML evaluation (nngp_gpfull_lml: build + Cholesky + -LML, the
work of one Nelder-Mead round of GPjax_p) at the shapes GParareal runs -- Burgers
N = 128 (1 152 points, rows up to 753), Hopf N = 512 (27 points, rows up to ~9 500), FHN-PDE
d_x = 10 (1 800 points, rows up to ~4 100) -- in every factor order (NNGP_GPF_ORDER / NNGP_GPF_FMA),
with the executed Cholesky rate (points x (rows+1)^3 / 3 flops per round) and the -LML agreement
between the orders.

    python tools/gpf_probe.py [rows:points ...]
"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nngp_amd as g  # noqa: E402
from nngp_amd import _lib  # noqa: E402

SHAPES = [(753, 1152), (378, 1152), (2048, 27), (4096, 240), (9500, 27)]
ORDERS = [('ll64', {'NNGP_GPF_ORDER': '0', 'NNGP_GPF_FMA': '0', 'NNGP_GPF_FUSE': '1'}),
          ('ll64_unfused', {'NNGP_GPF_ORDER': '0', 'NNGP_GPF_FMA': '0', 'NNGP_GPF_FUSE': '0'}),
          ('ll64_fma', {'NNGP_GPF_ORDER': '0', 'NNGP_GPF_FMA': '1', 'NNGP_GPF_FUSE': '1'}),
          ('rl32', {'NNGP_GPF_ORDER': '1', 'NNGP_GPF_FMA': '0'})]


def run(n, npts, d=3, reps=3):
    rng = np.random.default_rng(n)
    x = rng.uniform(-1, 1, (n, d))
    y = np.sin(2 * x) + 0.01 * rng.standard_normal((n, d))
    X = torch.tensor(x, device='cuda')
    Y = torch.tensor(y, device='cuda')
    c = np.ascontiguousarray(np.arange(npts) % d, dtype=np.int32)
    # GParareal's jitters (-20..-12) leave most of these matrices failing part-way (their later panels
    # are skipped, so the rate below would overstate the work); GPF_PROBE_JITTER=-2 makes every
    # factorisation complete, so executed = points x (rows+1)^3 / 3 exactly
    jit = os.environ.get('GPF_PROBE_JITTER')
    jx = np.ascontiguousarray(np.full(npts, float(jit)) if jit else -20.0 + (np.arange(npts) % 9), dtype=float)
    th = np.ascontiguousarray(np.column_stack([0.3 + 0.5 * rng.random(npts), 0.5 + rng.random(npts)]))
    fv = np.empty(npts)
    ip, dp = ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_double)
    out = {}
    only = os.environ.get('GPF_PROBE_ORDERS')
    for name, env in ORDERS:
        if only and name not in only.split(','):
            continue
        os.environ.update(env)
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            _lib.check(g.lib().nngp_gpfull_lml(X.data_ptr(), n, d, Y.data_ptr(), npts, c.ctypes.data_as(ip),
                                               jx.ctypes.data_as(dp), th.ctypes.data_as(dp), fv.ctypes.data_as(dp),
                                               None, None))
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        t = min(ts)
        fl = npts * (n + 1) ** 3 / 3
        out[name] = fv.copy()
        print(f'rows={n} points={npts} {name:9s}: {t * 1e3:9.2f} ms  {fl / t / 1e12:6.2f} TF/s executed Cholesky '
              f'({np.isfinite(fv).sum()} finite)', flush=True)
    if 'rl32' not in out:
        return
    ref = out['rl32']
    for name in [k for k in ('ll64', 'll64_fma') if k in out]:
        a = out[name]
        both = np.isfinite(a) & np.isfinite(ref)
        rel = np.abs(a[both] - ref[both]) / np.maximum(1, np.abs(ref[both])) if both.any() else np.zeros(1)
        print(f'   {name} vs rl32: finite pattern equal {np.array_equal(np.isfinite(a), np.isfinite(ref))}, '
              f'max rel diff {rel.max():.3g}, bitwise {np.mean(a[both] == ref[both]) if both.any() else 1:.3f}',
              flush=True)


if __name__ == '__main__':
    torch.cuda.set_device(0)
    shapes = [tuple(int(v) for v in a.split(':')) for a in sys.argv[1:]] or SHAPES
    for n, p in shapes:
        run(n, p)
