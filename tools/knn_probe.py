"""GPU probe: nngp_knn (distances + ordered top-m select only) at the Burgers training sizes."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nngp_amd as g  # noqa: E402

torch.cuda.set_device(0)
for rows in (127, 500, 1100, 3000):
    d, m = 128, 15
    X = torch.tensor(np.random.default_rng(rows).standard_normal((rows, d)), device='cuda')
    q = X[rows // 2] + 1e-3
    idx = torch.empty(m, dtype=torch.int32, device='cuda')
    dist = torch.empty(m, dtype=torch.float64, device='cuda')
    for _ in range(200):
        g._lib.check(g.lib().nngp_knn(X.data_ptr(), rows, d, q.data_ptr(), m, idx.data_ptr(), dist.data_ptr(), None))
    torch.cuda.synchronize()
    print('rows', rows, 'ok', flush=True)
