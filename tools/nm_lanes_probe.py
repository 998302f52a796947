"""GPU probe: throughput of one large batch of independent Nelder-Mead fits (Burgers-shaped: d = 128,
m = 15, every (coordinate, jitter) pair repeated with fresh theta0 draws) through nngp_nm_fit_batch,
on the 4-lanes-per-fit kernel (NNGP_NM_LANES=1) and on the packed 16-lane kernel (NNGP_NM_LANES=0).
Prints ms per batch and the batch's total Nelder-Mead evaluations (sum of nfev), so a PMC pass over
this program gives instructions per fit-evaluation.

    python tools/nm_lanes_probe.py [reps] [m] [copies] [modes]
      modes: comma-separated NNGP_NM_LANES[:NNGP_NM_LPF], e.g. "1:4,1:1,0" """
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nngp_amd as g  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    m = int(sys.argv[2]) if len(sys.argv) > 2 else 15
    copies = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    modes = (sys.argv[4] if len(sys.argv) > 4 else '1,0').split(',')
    torch.cuda.set_device(0)
    d = 128
    rng = np.random.default_rng(11)
    base = rng.uniform(-0.5, 0.5, size=d)
    xm = base + 0.05 * rng.standard_normal((m, d))
    ym = 0.01 * np.sin(3 * xm) + 1e-5 * rng.standard_normal((m, d))
    mdl = g.NNGP_p(n=d, N=4, nn=m, fatol=0.1, xatol=0.1, seed=7)
    coords = np.array([c for _ in range(copies) for c in range(d) for _ in range(9)], dtype=np.int32)
    jidx = np.array([j for _ in range(copies) for _ in range(d) for j in range(9)], dtype=np.int32)
    th0 = rng.integers(-8, 0, (len(coords), 2)).astype(np.float64)
    ref = None
    for mode in modes:
        lanes, _, lpf = mode.partition(':')
        os.environ['NNGP_NM_LANES'] = lanes
        os.environ['NNGP_NM_LPF'] = lpf or '4'
        res = mdl.fit_batch(xm, ym, coords, jidx, th0)   # warm-up (and the fits)
        if ref is None:
            ref = res
        same = (np.array_equal(res['theta'], ref['theta']) and np.array_equal(res['nfev'], ref['nfev']))
        times = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            mdl.fit_batch(xm, ym, coords, jidx, th0)
            b.record()
            b.synchronize()
            times.append(a.elapsed_time(b))
        ne = res['nfev'].astype(np.int64)
        print(f'NNGP_NM_LANES:LPF={mode} m={m}: {len(coords)} fits, {int(ne.sum())} evaluations '
              f'(mean {ne.mean():.1f}, max {ne.max()}), {min(times):.3f} ms per batch (incl. H2D/D2H), '
              f'{min(times) * 1e6 / ne.sum():.1f} ns per fit-evaluation; bitwise the first mode: {same}',
              flush=True)


if __name__ == '__main__':
    main()
