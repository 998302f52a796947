"""ctypes binding of libnngp_hip.so (include/nngp.h).

The product path has NO CPU fallback: if the HIP library is missing or no GPU is visible,
every compute entry point raises.  `lib()` loads the in-tree build
(nearest-neighbors-gparareal_amd/lib/libnngp_hip.so, produced by csrc/Makefile).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, 'lib', 'libnngp_hip.so')
CSRC = os.path.join(HERE, 'csrc')

# enums (include/nngp.h)
SYS_LORENZ, SYS_HOPF, SYS_THOMAS_LABYRINTH, SYS_FHN_ODE, SYS_ROSSLER = 0, 1, 2, 3, 4
SYS_BRUSSELATOR, SYS_DBL_PEND, SYS_BURGERS, SYS_FHN_PDE = 5, 6, 7, 8
TABLEAU = {'RK1': 1, 'RK2': 2, 'RK4': 4, 'RK8': 8}
STEP_FIXED, STEP_LINSPACE, STEP_CONTRACT = 0, 1, 16

EXPORTS = ['nngp_abi_version', 'nngp_last_error', 'nngp_device_count', 'nngp_rk_batch', 'nngp_rk_batch_grid',
           'nngp_rhs_batch', 'nngp_parareal_update', 'nngp_knn', 'nngp_nm_fit_batch',
           'nngp_gp_mean', 'nngp_predict', 'nngp_correction_sweep', 'nngp_gpfull_lml', 'nngp_gpfull_fit',
           'nngp_gpfull_mean', 'nngp_predict_range', 'nngp_chain_stats', 'nngp_sweep_late_reruns', 'nngp_shutdown',
           'nngp_comm_available', 'nngp_comm_unique_id', 'nngp_comm_init', 'nngp_comm_size', 'nngp_comm_destroy',
           'nngp_allgather_states', 'nngp_correction_sweep_sharded', 'nngp_correction_sweep_sharded_emulated']
MODEL_PARAREAL, MODEL_NNGP, MODEL_GPFULL = 0, 1, 2


class NNGPError(RuntimeError):
    pass


class CSystem(ctypes.Structure):
    """struct nngp_system"""
    _fields_ = [('kind', ctypes.c_int32), ('d', ctypes.c_int32), ('nx', ctypes.c_int32),
                ('normalized', ctypes.c_int32), ('param', ctypes.c_double * 4),
                ('norm', ctypes.c_void_p)]


_lib = None
_vp = ctypes.c_void_p
_dp = ctypes.POINTER(ctypes.c_double)


def build(force=False):
    """Compile csrc/ for gfx950 (hipcc cross-compiles without a GPU)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(['make', '-s', '-j3', '-C', CSRC], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NNGPError(f'HIP library not built: {LIB_PATH} missing (run __graft_entry__.build() or '
                        f'make -C {CSRC}); there is no CPU fallback')
    L = ctypes.CDLL(LIB_PATH)
    i32, i64, dbl = ctypes.c_int, ctypes.c_int64, ctypes.c_double
    L.nngp_abi_version.restype = i32
    L.nngp_last_error.restype = ctypes.c_char_p
    L.nngp_device_count.restype = i32
    L.nngp_rk_batch.argtypes = [ctypes.POINTER(CSystem), i32, i32, i32, _vp, _vp, i64, _vp, _vp, _vp]
    L.nngp_rk_batch_grid.argtypes = [ctypes.POINTER(CSystem), i32, i32, _vp, _vp, i64, _vp, i64, _vp, _vp, _vp]
    L.nngp_rhs_batch.argtypes = [ctypes.POINTER(CSystem), i32, _vp, _vp, _vp]
    L.nngp_parareal_update.argtypes = [i64, _vp, _vp, _vp, _vp, _vp]
    L.nngp_knn.argtypes = [_vp, i64, i32, _vp, i32, _vp, _vp, _vp]
    L.nngp_nm_fit_batch.argtypes = [i32, i32, _vp, _vp, i32, _vp, _vp, i32, _dp, _vp, dbl, dbl, i32,
                                    _vp, _vp, _vp, _vp]
    L.nngp_gp_mean.argtypes = [i32, i32, _vp, _vp, _vp, _vp, _vp, i32, _dp, _vp, _vp]
    L.nngp_predict.argtypes = [_vp, _vp, i64, i32, _vp, i32, i32, _dp, i32, _vp, dbl, dbl, i32, _vp,
                               _vp, _vp, _vp, _vp]
    L.nngp_correction_sweep.argtypes = [ctypes.POINTER(CSystem), i32, i32, i64, _vp, i32, i32, _vp, _vp, _vp,
                                        _vp, i32, _vp, _vp, i64, i32, i32, _dp, i32, _vp, dbl, dbl, i32,
                                        _vp, i32, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_float), _vp]
    _ip = ctypes.POINTER(ctypes.c_int32)
    L.nngp_gpfull_lml.argtypes = [_vp, i64, i32, _vp, i32, _ip, _dp, _dp, _dp, _vp, _vp]
    L.nngp_gpfull_fit.argtypes = [_vp, i64, i32, _vp, i32, _ip, _dp, _dp, dbl, dbl, i32, _dp, _dp, _ip, _ip, _vp]
    L.nngp_gpfull_mean.argtypes = [_vp, i64, i32, _vp, _vp, _vp, _vp, _vp, _vp]
    L.nngp_chain_stats.argtypes = [ctypes.POINTER(i64)]
    L.nngp_chain_stats.restype = i64
    L.nngp_sweep_late_reruns.argtypes = []
    L.nngp_sweep_late_reruns.restype = i64
    L.nngp_comm_available.argtypes = []
    L.nngp_comm_unique_id.argtypes = [ctypes.c_char_p]
    L.nngp_comm_init.argtypes = [i32, i32, ctypes.c_char_p]
    L.nngp_comm_size.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    L.nngp_comm_destroy.argtypes = []
    L.nngp_allgather_states.argtypes = [_vp, _vp, ctypes.c_size_t, _vp]
    L.nngp_correction_sweep_sharded.argtypes = [ctypes.POINTER(CSystem), i32, i32, i64, _vp, i32, i32, _vp, _vp,
                                                _vp, _vp, i64, i32, i32, _dp, i32, _vp, dbl, dbl, i32, _vp,
                                                ctypes.POINTER(ctypes.c_float), _vp]
    L.nngp_correction_sweep_sharded_emulated.argtypes = (L.nngp_correction_sweep_sharded.argtypes[:-2] +
                                                         [ctypes.c_size_t, i32, ctypes.POINTER(ctypes.c_float), _vp])
    L.nngp_predict_range.argtypes = [_vp, _vp, i64, i32, _vp, i32, i32, _dp, i32, _vp, i32, i32, dbl, dbl, i32,
                                     _vp, _vp]
    for name in EXPORTS:
        if name not in ('nngp_abi_version', 'nngp_last_error', 'nngp_device_count', 'nngp_chain_stats',
                        'nngp_sweep_late_reruns'):
            getattr(L, name).restype = i32
    if L.nngp_abi_version() != 1:
        raise NNGPError('ABI version mismatch')
    _lib = L
    return L


def check(rc):
    if rc != 0:
        msg = lib().nngp_last_error().decode(errors='replace')
        raise NNGPError(f'libnngp_hip error {rc}: {msg}')


def host_doubles(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a, a.ctypes.data_as(_dp)


_shutdown_registered = False


def require_gpu():
    """The product path runs on the GPU only; fail loudly otherwise.  The first call registers
    nngp_shutdown with atexit (it runs before torch's and the HIP runtime's own teardown)."""
    global _shutdown_registered
    import torch
    if not torch.cuda.is_available():
        raise NNGPError('no HIP device visible: nnGParareal-amd has no CPU fallback')
    L = lib()
    if not _shutdown_registered:
        import atexit
        atexit.register(L.nngp_shutdown)
        _shutdown_registered = True
    return torch


def as_device(a):
    """fp64 C-contiguous device tensor of a host array or a (device) tensor, without a copy when
    it already is one (the driver hands the models its device-resident training set)."""
    import torch
    if torch.is_tensor(a):
        return a.to(device='cuda', dtype=torch.float64).contiguous()
    return torch.tensor(np.ascontiguousarray(a, dtype=np.float64), device='cuda')


def chain_stats():
    """(fused-chain kernel launches, slices it completed) in this process (include/nngp.h)."""
    L = lib()
    sl = ctypes.c_int64(0)
    n = L.nngp_chain_stats(ctypes.byref(sl))
    return int(n), int(sl.value)


def sweep_late_reruns():
    """Sweeps rerun with the speculative batch serialised after a hit's wait timed out
    (include/nngp.h nngp_sweep_late_reruns), in this process."""
    return int(lib().nngp_sweep_late_reruns())


COMM_UID_BYTES = 128
_comm_state = {'group': None, 'key': None}


def comm_release():
    """Release the library's communicator (nngp_comm_destroy) and forget which group it served."""
    _comm_state.update(group=None, key=None)
    if _lib is not None:
        _lib.nngp_comm_destroy()


def comm_for(group=None):
    """The library's RCCL communicator (include/nngp.h nngp_comm_*) over the torch.distributed
    `group`, created once per group: rank 0 makes the unique id, torch broadcasts it, every rank
    joins on its current device.  Returns True when the native collectives are live for `group`;
    False for a gloo group (ranks sharing one GPU: RCCL refuses duplicate devices) or when RCCL
    cannot be loaded, or the init fails, on some rank -- the caller then keeps torch.distributed's
    collectives.  Collective: every rank of `group` must call it together.

    Every decision is a MIN all-reduce over the ranks, so they all take the same branch:
    - the cache (this group's communicator is live on this rank) -- a rank that released its
      communicator (nngp_shutdown / nngp_comm_destroy) makes every rank re-create it;
    - RCCL resolvable on every rank (nngp_comm_available) and rank 0's id created: only rank 0
      calls nngp_comm_unique_id, which starts RCCL's bootstrap listener;
    - every rank's init succeeded (nngp_comm_init: non-blocking init with a deadline,
      NNGP_COMM_TIMEOUT_S, so a missing peer ends in an error on that rank, not a hang)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_backend(group) != 'nccl':
        return False
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    gobj = group if group is not None else dist.group.WORLD
    key = (id(gobj), world, rank)
    L = lib()

    def agree(ok):   # MIN over the group's ranks
        flag = torch.tensor([int(ok)], dtype=torch.int32, device='cuda')
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
        return int(flag.item())

    # 1: this group's communicator is live here; 0: not created / released; -1: the watchdog
    # aborted it (a collective ran past the deadline, so results since then are void) -> raise
    state = 0
    if _comm_state['key'] == key and _comm_state['group'] is gobj:
        nr, rk = ctypes.c_int(0), ctypes.c_int(-1)
        rc = L.nngp_comm_size(ctypes.byref(nr), ctypes.byref(rk))
        state = -1 if rc != 0 else int((nr.value, rk.value) == (world, rank))
    state = agree(state)
    if state < 0:
        _comm_state.update(group=None, key=None)
        raise NNGPError('the library communicator was aborted on some rank: a collective ran past '
                        'NNGP_COMM_TIMEOUT_S (' + L.nngp_last_error().decode(errors='replace') + ')')
    if state == 1:
        return True
    _comm_state.update(group=None, key=None)
    L.nngp_comm_destroy()   # every rank starts the re-creation from no communicator
    uid = ctypes.create_string_buffer(COMM_UID_BYTES)
    ok = L.nngp_comm_available() == 0
    if ok and rank == 0:
        ok = L.nngp_comm_unique_id(uid) == 0
    if agree(ok) != 1:
        return False
    obj = [uid.raw]
    src = 0 if group is None else dist.get_global_rank(group, 0)
    dist.broadcast_object_list(obj, src=src, group=group)
    rc = L.nngp_comm_init(world, rank, obj[0])
    if agree(rc == 0) != 1:
        L.nngp_comm_destroy()
        return False
    _comm_state.update(group=gobj, key=key)
    return True
