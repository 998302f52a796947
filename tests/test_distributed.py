"""CPU, multi-process: the N>1 fine-sweep sharding over `gloo`.

Each rank integrates its contiguous block of the unconverged slices with one batched call and a
single all-gather reassembles U_F in slice order on every rank.  The propagator here is the CPU
oracle's batched RK (a test double standing in for the HIP launch, which needs a GPU); the
sharding, padding and gather are the product code (parareal.fine_sweep_sharded)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle as O


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cases, q):
    import torch
    import torch.distributed as dist
    import nngp_amd
    from nngp_amd.parareal import fine_sweep_sharded
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        so = O.System('lorenz')
        calls = []

        def propagate(t0, t1, U0, out):
            calls.append(U0.shape[0])
            out.copy_(torch.from_numpy(so.rk_batch(4, t0.numpy(), t1.numpy(), 45, U0.numpy())))

        res = []
        for N, I in cases:
            rng = np.random.default_rng(N * 100 + I)
            t = torch.from_numpy(np.linspace(0, 18, N + 1))
            U = torch.from_numpy(rng.uniform(-0.5, 0.5, (N + 1, 3)))
            UF = torch.full((N + 1, 3), float('nan'), dtype=torch.float64)
            fine_sweep_sharded(propagate, t, U, UF, I, N)
            res.append(UF.numpy().copy())
        q.put((rank, res, calls))
    finally:
        dist.destroy_process_group()


CASES = [(8, 0), (8, 3), (7, 1), (5, 4), (16, 2)]


@pytest.mark.parametrize('world', [2, 3])
def test_sharded_fine_sweep_equals_single_process(world):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, CASES, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort(key=lambda r: r[0])
    so = O.System('lorenz')
    for c, (N, I) in enumerate(CASES):
        rng = np.random.default_rng(N * 100 + I)
        t = np.linspace(0, 18, N + 1)
        U = rng.uniform(-0.5, 0.5, (N + 1, 3))
        ref = so.rk_batch(4, t[I:N], t[I + 1:N + 1], 45, U[I:N])
        for rank, res, _ in out:
            got = res[c]
            assert np.all(np.isnan(got[:I + 1]))            # untouched rows stay untouched
            assert np.array_equal(got[I + 1:], ref), (world, rank, N, I)
    # every rank launched at most one batched propagation per sweep, blocks of ceil((N-I)/world)
    for rank, _, calls in out:
        assert all(n <= max((N - I + world - 1) // world for N, I in CASES) for n in calls)


@pytest.mark.parametrize('world', [1, 2, 3, 4, 8])
def test_shard_bounds_partition_the_unconverged_slices(world):
    from nngp_amd.parareal import shard_bounds
    for N in (1, 2, 7, 32, 128, 513):
        for I in range(0, N, max(1, N // 7)):
            blocks = [shard_bounds(I, N, world, r) for r in range(world)]
            chunk = blocks[0][2]
            covered = []
            for lo, hi, ch in blocks:
                assert ch == chunk and 0 <= hi - lo <= chunk
                covered.extend(range(lo, hi))
            assert covered == list(range(I, N))                 # contiguous, ordered, complete
            assert world * chunk >= N - I


# ------------------------------------------------ correction sweep sharded by coordinate (§8e)
def _sweep_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    import nngp_amd  # noqa: F401
    from nngp_amd.parareal import correction_sweep_sharded
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        args = _sweep_case()
        calls = []

        def predict_range(i, c0, c1, u, out):
            calls.append((c0, c1))
            out.copy_(torch.from_numpy(_oracle_preds(args, i, u.numpy())[c0:c1]))

        U1, UG1 = _run_sweep(args, lambda co, pr, asm, I, N, U1, UG1, d: correction_sweep_sharded(
            co, pr, asm, I, N, U1, UG1, d), predict_range)
        q.put((rank, U1.numpy().copy(), UG1.numpy().copy(), sorted(set(calls))))
    finally:
        dist.destroy_process_group()


def _sweep_case():
    so = O.System('lorenz')
    rng = np.random.default_rng(5)
    N, I, d = 6, 1, 3
    X = rng.uniform(-0.5, 0.5, (40, d))
    Y = 1e-3 * np.sin(3 * X)
    th0 = rng.integers(-8, 0, ((N - I) * d * 9, 2)).astype(float)
    t = np.linspace(0, 18, N + 1)
    U1 = np.full((N + 1, d), np.nan)
    U1[I] = rng.uniform(-0.5, 0.5, d)
    return dict(so=so, N=N, I=I, d=d, X=X, Y=Y, th0=th0, t=t, U1=U1)


def _oracle_preds(a, i, u):
    j = i - a['I']
    nf = a['d'] * 9
    return O.predict(a['X'], a['Y'], u, 10, a['th0'][j * nf:(j + 1) * nf])


def _run_sweep(a, sweep, predict_range):
    import torch
    U1 = torch.from_numpy(a['U1'].copy())
    UG1 = torch.full_like(U1, float('nan'))

    def coarse(i, u, out):
        out.copy_(torch.from_numpy(a['so'].rk_batch(4, a['t'][i:i + 1], a['t'][i + 1:i + 2], 6, u.numpy()[None])[0]))

    def assemble(preds, ug, out):
        out.copy_((preds - 0.0) + ug)

    sweep(coarse, predict_range, assemble, a['I'], a['N'], U1, UG1, a['d'])
    return U1, UG1


@pytest.mark.parametrize('world', [2, 3])
def test_sharded_correction_sweep_equals_unsharded(world):
    """Each rank predicts only its coordinate block; one all-gather per slice reassembles the
    prediction; every rank ends with the unsharded sweep's iterates bit for bit."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sweep_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    a = _sweep_case()

    def serial(co, pr, asm, I, N, U1, UG1, d):
        import torch
        for i in range(I, N):
            co(i, U1[i], UG1[i + 1])
            p_ = torch.empty(d, dtype=torch.float64)
            pr(i, 0, d, U1[i], p_)
            asm(p_, UG1[i + 1], U1[i + 1])

    import torch
    refU, refG = _run_sweep(a, serial, lambda i, c0, c1, u, o: o.copy_(
        torch.from_numpy(_oracle_preds(a, i, u.numpy())[c0:c1])))
    blocks = set()
    for rank, U1, UG1, calls in out:
        assert np.array_equal(np.nan_to_num(U1, nan=7.0), np.nan_to_num(refU.numpy(), nan=7.0)), rank
        assert np.array_equal(np.nan_to_num(UG1, nan=7.0), np.nan_to_num(refG.numpy(), nan=7.0)), rank
        blocks.update(calls)
    assert sorted(blocks) == sorted({(lo, hi) for lo, hi in
                                     [(min(r * -(-3 // world), 3), min((r + 1) * -(-3 // world), 3))
                                      for r in range(world)] if hi > lo})
