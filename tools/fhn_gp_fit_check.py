"""FHN-PDE d_x = 10 GParareal: the GPU's selected hyperparameters after the
first training call of the published-configuration run, against the CPU oracle's (oracle/gpfull.py:
numpy/LAPACK Cholesky + scipy Nelder-Mead, the reference's own algorithm) on the same training set
(rows 0..511 of the run's store_int dump) for the first coordinates.

    python tools/fhn_gp_fit_check.py <dump.npz> [n_coords]"""
import json
import os
import sys

os.environ.setdefault('OMP_NUM_THREADS', '1')       # one BLAS thread per worker process
os.environ.setdefault('OPENBLAS_NUM_THREADS', '1')
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'oracle')]
import gpfull as GF  # noqa: E402
from nngp_amd.models import JITTERS, _select_fit  # noqa: E402


def coord_fits(args):
    x, y, j = args
    out = [GF.gp_fit(x, y, np.array([1.0, 1.0]), jit, 1e-4, 1e-4) for jit in JITTERS]
    print(f'coord {j} done', flush=True)
    th = np.array([o[0] for o in out])
    fv = np.array([o[1] for o in out])
    return j, th, fv, [o[2] for o in out]


def main():
    z = np.load(sys.argv[1], allow_pickle=False)
    nc = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    meta = json.loads(str(z['meta']))
    hyp = np.array(meta['model']['hyp'])
    x, D = z['x'][:512], z['D'][:512]
    with ProcessPoolExecutor(min(nc, 8)) as ex:
        for j, th, fv, ne in ex.map(coord_fits, [(x, D[:, j], j) for j in range(nc)]):
            p, f, jit = _select_fit(th, fv, JITTERS)
            print(f'coord {j}: oracle theta {np.round(p, 6).tolist()} -LML {f:.6g} jitter {jit} nfev {ne} | '
                  f'GPU theta {np.round(hyp[j, :, 1], 6).tolist()}', flush=True)


if __name__ == '__main__':
    main()
