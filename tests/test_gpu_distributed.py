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
                                              ('fhn', '1', 2), ('tomlab256', 'none', 8), ('fhn800', '1', 8),
                                              ('gp_burgers', 'none', 2), ('gp_burgers', 'none', 3)])
def test_multi_rank_gpu_run_equals_single_rank(gpu, case, shard, world, tmp_path):
    """world 8: BASELINE configs[3] / configs[4]'s 8-way partitions (TomLab N=256: 32 slices per
    rank; FHN-PDE d=800 N=512: 64 slices and 100 of the 800 coordinates per rank).  gp_burgers:
    GParareal's d*9 = 576 fits and its 64 posterior-weight vectors sharded by coordinate (32 / 32
    and 22 / 22 / 20 per rank), one all-gather each per iteration (models.GPjax_p._train/_weights)."""
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


@pytest.mark.timeout(300)
def test_native_rccl_comm_and_sharded_sweep_one_rank(gpu, tmp_path):
    """The C-ABI's multi-GPU exchange on the box's one GPU: an NCCL (RCCL) process group of one
    rank, the library's communicator created from it (_lib.comm_for), nngp_allgather_states, and
    nngp_correction_sweep_sharded (every slice's G, this rank's coordinates, the RCCL all-gather and
    u = preds + uG issued natively) -- bitwise the unsharded run, with and without the native path,
    and with the coordinate split of 3, 7 and 8 ranks played in turn by the one process
    (NNGP_SHARD_EMULATE_RANKS -> nngp_correction_sweep_sharded_emulated: each rank's block and the
    partial last one land where the in-place all-gather would put them; a gather buffer shorter than
    the split is refused before any launch).
    Several ranks need several GPUs for RCCL (the 8-GPU bench runs them); the orchestration across
    ranks is covered on gloo above."""
    out = str(tmp_path / 'comm.npz')
    code = r'''
import os, sys, socket
import numpy as np
import torch
sys.path.insert(0, os.environ["NNGP_ROOT"]); sys.path.insert(0, os.path.join(os.environ["NNGP_ROOT"], "tests"))
torch.cuda.set_device(0)
with socket.socket() as s:
    s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]
torch.distributed.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                     device_id=torch.device("cuda", 0))
import nngp_amd as g
from nngp_amd import _lib
from dist_gpu_worker import run_case
assert _lib.comm_for(None)
L = _lib.lib()
import ctypes
nr, rk = ctypes.c_int(0), ctypes.c_int(0)
L.nngp_comm_size(ctypes.byref(nr), ctypes.byref(rk))
assert (nr.value, rk.value) == (1, 0)
x = torch.arange(10, dtype=torch.float64, device="cuda"); y = torch.zeros(10, dtype=torch.float64, device="cuda")
_lib.check(L.nngp_allgather_states(x.data_ptr(), y.data_ptr(), 10, torch.cuda.current_stream().cuda_stream))
torch.cuda.synchronize(); assert torch.equal(x, y)
k0, c0, u0 = run_case(g, "fhn", None)          # unsharded (world 1)
k1, c1, u1 = run_case(g, "fhn", True, native=True)   # native sharded sweep
same = lambda a, b: bool(np.array_equal(np.nan_to_num(a, nan=7.0), np.nan_to_num(b, nan=7.0)))
# the coordinate split of W ranks played in turn by this process (NNGP_SHARD_EMULATE_RANKS): every
# rank's [c0, c1) into its block of the gather buffer, the partial last block included (d = 200:
# W = 3 -> blocks of 67, 67, 66; W = 7 -> 29 x 6 + 26; W = 8 -> 25 x 8)
emu = []
for W in (3, 7, 8):
    os.environ["NNGP_SHARD_EMULATE_RANKS"] = str(W)
    kw_, cw_, uw_ = run_case(g, "fhn", True, native=True)
    emu.append(kw_ == k0 and list(cw_) == list(c0) and same(uw_, u0))
del os.environ["NNGP_SHARD_EMULATE_RANKS"]
# the emulated entry checks the caller's gather length (3 ranks x 67 > 200) before launching
ode = g.FHN_PDE(d_x=10)
cs = ode.get_vector_field().csystem(torch.device("cuda", 0))
buf = torch.zeros((17, 200), dtype=torch.float64, device="cuda")
short = torch.zeros(200, dtype=torch.float64, device="cuda")
jit = np.arange(-20, -11, dtype=float)
rc_short = L.nngp_correction_sweep_sharded_emulated(
    ctypes.byref(cs), 4, 0, 5, buf.data_ptr(), 0, 1, buf.data_ptr(), buf.data_ptr(), buf.data_ptr(), buf.data_ptr(),
    16, 10, 9, jit.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), 1, buf.data_ptr(), 0.1, 0.1, 400,
    short.data_ptr(), short.numel(), 3, None, torch.cuda.current_stream().cuda_stream)
assert rc_short == -1 and b"gather holds" in L.nngp_last_error(), (rc_short, L.nngp_last_error())
s = g.SolverRK(ode.get_vector_field(), Ng=5, Nf=100, F="RK8", G="RK4")
r2 = g.Parareal(ode, s, [0, 8], 16, epsilon=5e-7, verbose=None).run(model="nngp", nn=20, seed=45, early_stop=2,
                                                                  shard_corrections=True, native_comm=False)
np.savez(sys.argv[1], k=[k0, k1, r2["k"]], same_native=np.array_equal(np.nan_to_num(u0, nan=7.0), np.nan_to_num(u1, nan=7.0)),
         emulated=np.array(emu),
         same_py=np.array_equal(np.nan_to_num(u0, nan=7.0), np.nan_to_num(r2["u"], nan=7.0)),
         conv=[list(c0) == list(c1), list(c0) == list(r2["conv_int"])])
torch.distributed.destroy_process_group()
print("comm ok")
'''
    root = os.path.dirname(HERE)
    p = subprocess.run([sys.executable, '-c', code, out], env=dict(os.environ, NNGP_ROOT=root),
                       capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-3000:])
    R = np.load(out)
    assert len(set(R['k'].tolist())) == 1 and bool(R['same_native']) and bool(R['same_py']) and all(R['conv'])
    assert R['emulated'].tolist() == [True, True, True], R['emulated']


@pytest.mark.timeout(120)
def test_comm_init_without_peers_returns_in_bounded_time(gpu):
    """The communicator's deadline (include/nngp.h, NNGP_COMM_TIMEOUT_S): a rank that joins a
    two-rank communicator whose peer never arrives gets NNGP_E_HIP after the deadline (RCCL's
    non-blocking init, polled, then ncclCommAbort) instead of blocking forever -- and the library
    creates a working communicator afterwards.  Run in a child process under its own limit."""
    code = r'''
import ctypes, os, sys, time
import torch
sys.path.insert(0, os.environ["NNGP_ROOT"])
torch.cuda.set_device(0)
from nngp_amd import _lib
L = _lib.lib()
uid = ctypes.create_string_buffer(_lib.COMM_UID_BYTES)
assert L.nngp_comm_available() == 0
assert L.nngp_comm_unique_id(uid) == 0
t0 = time.time()
rc = L.nngp_comm_init(2, 0, uid.raw)
el = time.time() - t0
msg = L.nngp_last_error().decode()
print("init without a peer: rc", rc, "after", round(el, 1), "s:", msg, flush=True)
assert rc == -2 and "still waiting for its peers" in msg and el < 40, (rc, el, msg)
nr, rk = ctypes.c_int(7), ctypes.c_int(7)
assert L.nngp_comm_size(ctypes.byref(nr), ctypes.byref(rk)) == 0 and (nr.value, rk.value) == (0, -1)
# a one-rank communicator works after the aborted one
assert L.nngp_comm_unique_id(uid) == 0
assert L.nngp_comm_init(1, 0, uid.raw) == 0, L.nngp_last_error()
x = torch.arange(6, dtype=torch.float64, device="cuda"); y = torch.zeros(6, dtype=torch.float64, device="cuda")
_lib.check(L.nngp_allgather_states(x.data_ptr(), y.data_ptr(), 6, torch.cuda.current_stream().cuda_stream))
torch.cuda.synchronize(); assert torch.equal(x, y)
assert L.nngp_comm_destroy() == 0
print("deadline ok", flush=True)
'''
    root = os.path.dirname(HERE)
    p = subprocess.run([sys.executable, '-c', code], env=dict(os.environ, NNGP_ROOT=root, NNGP_COMM_TIMEOUT_S='5'),
                       capture_output=True, text=True, timeout=100)
    print(p.stdout[-1500:])
    assert p.returncode == 0 and 'deadline ok' in p.stdout, (p.stdout[-2000:], p.stderr[-3000:])
