"""Where a run's wall-clock goes between kernels: from a rocprofv3 --kernel-trace CSV
(*_kernel_trace.csv), the busy time (union of all dispatch intervals), the idle gaps between
them, and the largest gaps with the kernels either side.  Usage:
    python tools/timeline_gaps.py <kernel_trace.csv> [t_from_s] [t_to_s]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'][:60]) for r in rows)
    t0 = ev[0][0]
    lo = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
    hi = float(sys.argv[3]) if len(sys.argv) > 3 else 1e30
    ev = [e for e in ev if lo <= (e[0] - t0) / 1e9 <= hi]
    busy, gaps, end, last = 0, [], None, None
    for s, e, n in ev:
        if end is None or s > end:
            if end is not None:
                gaps.append((s - end, last, n, (end - t0) / 1e9))
            busy += e - s
            end = e
        else:
            if e > end:
                busy += e - end
                end = e
        last = n
    span = ev[-1][1] - ev[0][0]
    print(f'dispatches {len(ev)}  span {span / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  idle {(span - busy) / 1e6:.3f} ms '
          f'in {len(gaps)} gaps')
    for g, a, b, at in sorted(gaps, reverse=True)[:25]:
        print(f'  {g / 1e3:9.1f} us at {at:9.4f} s  after {a}  before {b}')


if __name__ == '__main__':
    main()
