"""PMC attribution probe for the fine kernel's HBM traffic (run under rocprofv3 --pmc, one counter
set per pass; tools/gpu_r3_pmc.sh).

The TCC counters behind FETCH_SIZE / WRITE_SIZE are device-wide: a multi-second launch also
collects whatever else reaches the memory side of the L2 in that window.  This probe alternates
the bench's fine sweep (rk_group_kernel<HOPF,RK4>, 128 slices, the headline launch) with a
null kernel of the same duration that writes nothing (torch.cuda._sleep: a spin on the clock),
and runs short launches of the fine kernel too, so the per-dispatch counter rows show which bytes
belong to the kernel (constant per launch, independent of its duration) and which to the window
(present in the null kernel as well, growing with the duration).
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import nngp_amd as g  # noqa: E402


def main():
    torch.cuda.set_device(0)
    long_steps = 2048 * 85 * 10000 // 128          # the headline schedule: ~2.7 s per launch
    n = 128
    rng = np.random.default_rng(1234)
    t = np.linspace(-20, 500, n + 1)
    U = rng.uniform(-0.5, 0.5, size=(n, 3))
    dev = lambda a: torch.tensor(a, dtype=torch.float64, device='cuda')
    t0, t1, u0 = dev(t[:n]), dev(t[1:]), dev(U)
    out = torch.empty_like(u0)
    solver_long = bench.hopf_setup(g, long_steps, n)[1]
    solver_short = bench.hopf_setup(g, 10000, n)[1]
    torch.cuda.synchronize()
    # the null kernel's spin count for one long launch's duration, calibrated on the box
    a = time.perf_counter()
    solver_long.run_F_batch(t0, t1, u0, out=out)
    torch.cuda.synchronize()
    dur = time.perf_counter() - a
    a = time.perf_counter()
    torch.cuda._sleep(100_000_000)
    torch.cuda.synchronize()
    rate = 100_000_000 / (time.perf_counter() - a)
    cycles = int(min(dur, 5.0) * rate)
    print(f'long launch {dur:.3f} s; null kernel {rate:.3e} cycles/s -> {cycles} cycles', flush=True)
    if len(sys.argv) > 2 and sys.argv[1] == 'null':   # many null windows only (the background's rate)
        for i in range(int(sys.argv[2])):
            torch.cuda._sleep(cycles)
            torch.cuda.synchronize()
        print('done', flush=True)
        return
    for i in range(4):
        solver_long.run_F_batch(t0, t1, u0, out=out)
        torch.cuda.synchronize()
        torch.cuda._sleep(cycles)
        torch.cuda.synchronize()
    for i in range(8):
        solver_short.run_F_batch(t0, t1, u0, out=out)
        torch.cuda.synchronize()
    print('done', flush=True)


if __name__ == '__main__':
    main()
