"""GPU probe: FHN-PDE N=512 fine sweep (d=200 published schedule, d=800) per step at each
NNGP_RK_THREADS (threads per slice; combinations beyond the field kernel's 8 elements per thread
are skipped)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import nngp_amd as g  # noqa: E402

torch.cuda.set_device(0)
for thr in ('64', '128', '192', '256', '320', '384', '448', '512', '832', '1024'):
    os.environ['NNGP_RK_THREADS'] = thr
    try:
        r = bench.fhn_pde_fine_sweeps(torch, g)
        print(thr, {k: round(v['us_per_step'], 3) for k, v in r.items()}, flush=True)
    except g.NNGPError as e:
        print(thr, 'skipped:', e, flush=True)
