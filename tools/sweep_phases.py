"""Per-iteration phases of a Burgers nnGParareal run from a rocprofv3 --kernel-trace CSV: the F
launch, the overlapped batch, and the correction sweep slice by slice (G -> kNN distance ->
select -> [fits] -> mean), with the sweep's time split into hit slices and missed slices.
    python tools/sweep_phases.py <kernel_trace.csv> [run_index]
A run is a group of iterations whose F launches are < 1 s apart; the default is the last run."""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in rows)
    isF = lambda n: 'rk_burgers_wave_kernel<8' in n
    isG = lambda n: 'rk_burgers_wave_kernel<1' in n
    Fs = [e for e in ev if isF(e[2])]
    runs, cur = [], [Fs[0]]
    for a, b in zip(Fs, Fs[1:]):
        if b[0] - a[1] > 1e9:
            runs.append(cur)
            cur = []
        cur.append(b)
    runs.append(cur)
    run = runs[int(sys.argv[2]) if len(sys.argv) > 2 else -1]
    print(f'{len(runs)} runs; run with {len(run)} iterations')
    for it, f in enumerate(run):
        t0 = f[0]
        t1 = run[it + 1][0] if it + 1 < len(run) else t0 + int(1e9)
        k = [e for e in ev if t0 <= e[0] < t1]
        end = max(e[1] for e in k)
        batch = [e for e in k if 'nm_lane_kernel' in e[2] or 'nm_fit_kernel' in e[2]]
        b_end = max((e[1] for e in batch), default=t0)
        gs = [e for e in k if isG(e[2])]
        means = [e for e in k if 'gp_mean_kernel' in e[2]]
        # slice i: from its G start to the next slice's G start (the last: to its mean's end)
        hit_t, miss_t, nh, nm = 0, 0, 0, 0
        after_batch = 0
        for s, g in enumerate(gs):
            nxt = gs[s + 1][0] if s + 1 < len(gs) else end
            fits = [e for e in k if g[0] <= e[0] < nxt and ('nm_spec' in e[2]) and e[0] > b_end]
            fits_any = [e for e in k if g[0] <= e[0] < nxt and 'nm_spec' in e[2]]
            dt = nxt - g[0]
            if fits_any:
                miss_t += dt
                nm += 1
            else:
                hit_t += dt
                nh += 1
            if g[0] >= b_end:
                after_batch += 1
        print(f'iter {it}: {(end - t0) / 1e6:7.2f} ms  F {(f[1] - f[0]) / 1e6:5.2f}  batch ends {(b_end - t0) / 1e6:6.2f}  '
              f'sweep {len(gs)} slices ({after_batch} start after the batch): {nh} without fits {hit_t / 1e6:6.2f} ms '
              f'({hit_t / max(nh, 1) / 1e3:5.1f} us each), {nm} with fits launched {miss_t / 1e6:6.2f} ms '
              f'({miss_t / max(nm, 1) / 1e3:6.1f} us each)')


if __name__ == '__main__':
    main()
