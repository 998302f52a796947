"""GPU probe: timing of one nnGP correction (fused predict) at Hopf / Burgers / FHN shapes, and the
distribution of Nelder-Mead evaluation counts (the kernel's latency driver)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nngp_amd as g  # noqa: E402


def case(d, m, R, rows, seed=0):
    rng = np.random.default_rng(seed)
    base = rng.uniform(-0.5, 0.5, size=d)
    # trajectory-like training set: a random walk of states, smooth targets
    X = base + np.cumsum(0.02 * rng.standard_normal((rows, d)), axis=0)
    Y = 0.01 * np.sin(3 * X) + 1e-5 * rng.standard_normal((rows, d))
    q = X[rows // 2] + 0.005
    mdl = g.NNGP_p(n=d, N=8, nn=m, n_restarts=R, seed=seed)
    dev = lambda a: torch.tensor(a, dtype=torch.float64, device='cuda')
    Xd, Yd, qd = dev(X), dev(Y), dev(q)
    th = dev(mdl.draw_thetas(1))
    fits = torch.empty((mdl.n_fits, 4), dtype=torch.float64, device='cuda')
    for _ in range(2):
        mdl.predict_device(Xd, Yd, rows, qd, th, fits_out=fits)
    torch.cuda.synchronize()
    reps = 5
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        mdl.predict_device(Xd, Yd, rows, qd, th, fits_out=fits)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    nfev = fits[:, 3].cpu().numpy()
    print(f'd={d:4d} m={m} R={R} rows={rows}: {ms:8.3f} ms/correction  fits={mdl.n_fits}  '
          f'nfev mean {nfev.mean():.0f} p90 {np.percentile(nfev, 90):.0f} max {nfev.max():.0f} '
          f'-> {ms * 1e3 / nfev.max():.1f} us per eval at the slowest fit', flush=True)


if __name__ == '__main__':
    torch.cuda.set_device(0)
    if len(sys.argv) > 1 and sys.argv[1] == 'sweep':
        # spec-vs-packed crossover (run once with NNGP_NM_SPEC=1 and once with 0)
        for m, ds in ((15, (64, 96, 128, 160, 192, 256)), (20, (32, 64, 96, 128, 160, 200)),
                      (30, (16, 32, 64, 96))):
            for d in ds:
                case(d, m, 1, 1500)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == 'level2':
        # latency-bound corrections (run with NNGP_NM_LEVEL2=0 / 1 / 2 / 4)
        case(3, 15, 2, 600)
        case(3, 10, 1, 600)
        case(2, 15, 2, 600)
        case(20, 20, 1, 1500)
        case(40, 15, 1, 1500)
        case(100, 20, 1, 3000)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == 'park':
        # packed-kernel shapes (run with NNGP_NM_PARK=0 / 60 / 100 / 150)
        case(256, 15, 1, 1500)
        case(400, 15, 1, 2000)
        case(200, 20, 1, 3000)
        case(800, 20, 1, 4000)
        sys.exit(0)
    case(3, 15, 2, 600)
    case(3, 10, 1, 600)
    case(128, 15, 1, 1200)
    case(200, 20, 1, 3000)
    case(800, 20, 1, 4000)
