"""Largest dispatches of one kernel in a rocprofv3 --pmc counter_collection.csv (one counter per pass
for FETCH_SIZE / WRITE_SIZE): per dispatch the grid, duration and counter value, the N longest.
    python tools/pmc_dispatch_top.py <counter_collection.csv> [SUBSTRING] [N]"""
import csv
import sys


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ''
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    per = {}
    for r in csv.DictReader(open(path)):
        if sub not in r.get('Kernel_Name', ''):
            continue
        d = per.setdefault(r['Dispatch_Id'], {'grid': int(r.get('Grid_Size', 0)), 'counters': {},
                                               'ns': int(r['End_Timestamp']) - int(r['Start_Timestamp'])})
        d['counters'][r['Counter_Name']] = d['counters'].get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    rows = sorted(per.items(), key=lambda kv: -kv[1]['ns'])[:n]
    tot = {}
    for _, d in per.items():
        for c, v in d['counters'].items():
            tot[c] = tot.get(c, 0.0) + v
    print(f'{len(per)} dispatches; totals {tot}; total ns {sum(d["ns"] for d in per.values())}')
    for k, d in rows:
        print(f'dispatch {k} grid {d["grid"]} {d["ns"] / 1e3:.1f} us {d["counters"]}')


if __name__ == '__main__':
    main()
