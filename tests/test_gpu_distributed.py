"""Multi-rank orchestration WITH the HIP path (tests/test_distributed.py covers it on CPU with the
oracle as propagator): 2, 3 and 8 ranks in a gloo group share the box's one GPU (RCCL refuses
duplicate devices; gloo stages the all-gathers through host memory), each running the native
kernels -- the fine sweep sharded into contiguous slice blocks and, for FHN-PDE, every
prediction's fits sharded by coordinate (nngp_predict_range).  The iterates, K and conv_int must
equal the single-rank run's bit for bit (parareal.py's replicated sweep keeps ranks identical)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from dist_gpu_worker import run_case

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.mark.timeout(400)
@pytest.mark.parametrize('case,shard,world', [('lorenz', 'none', 2), ('burgers', 'none', 2), ('burgers', '1', 3),
                                              ('fhn', '1', 2), ('tomlab256', 'none', 8), ('fhn800', '1', 8)])
def test_multi_rank_gpu_run_equals_single_rank(gpu, case, shard, world, tmp_path):
    """world 8: BASELINE configs[3] / configs[4]'s 8-way partitions (TomLab N=256: 32 slices per
    rank; FHN-PDE d=800 N=512: 64 slices and 100 of the 800 coordinates per rank)."""
    k1, conv1, u1 = run_case(gpu, case, None if shard == 'none' else shard == '1')
    out = str(tmp_path / 'rank0.npz')
    port = _port()
    procs = []
    for rank in range(world):
        env = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                   WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, 'dist_gpu_worker.py'), case, out, shard],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=300)[0].decode(errors='replace'))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert all(p.returncode == 0 for p in procs), '\n'.join(l[-2000:] for l in logs)
    R = np.load(out)
    assert int(R['k']) == k1 and list(R['conv']) == list(conv1)
    assert np.array_equal(np.nan_to_num(R['u'], nan=7.0), np.nan_to_num(u1, nan=7.0))
