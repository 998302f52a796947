"""Per-dispatch HBM traffic of the fine kernel from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of
tools/pmc_probe.py (one counter per pass, tools/gpu_r3_b.sh).

FETCH_SIZE / WRITE_SIZE are in KiB and count the L2's memory-side requests of the whole device
while a dispatch runs.  MI355X_MICROARCH.md (HBM section): on gfx950 FETCH_SIZE reports 1/2 of the
bytes of wide coalesced streaming reads, so the reported fetch is FETCH_SIZE x 2 (raw beside it);
WRITE_SIZE is taken as is.  Every dispatch of both passes is listed, with its kernel and duration:
the fine kernel's long launches (the bench's headline launch), its short launches (same bytes,
~0.1 % of the duration) and the null kernel (torch.cuda._sleep, no memory traffic of its own)
of the same duration as a long launch -- what the null kernel shows is the device's background
during such a window, not the fine kernel's.

Usage: python tools/pmc_traffic.py <fetch.csv> <write.csv> <out.json> [kernel-substring]
"""
import csv
import json
import statistics
import sys


def rows(path):
    out = []
    for r in csv.DictReader(open(path)):
        out.append({'dispatch': int(r['Dispatch_Id']), 'kernel': r['Kernel_Name'],
                    'ms': (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6,
                    'bytes': float(r['Counter_Value']) * 1024.0})
    return sorted(out, key=lambda x: x['dispatch'])


def classify(k, sub, long_ms):
    if sub in k['kernel']:
        return 'fine_long' if k['ms'] > 0.5 * long_ms else 'fine_short'
    if 'sleep' in k['kernel'].lower() or 'spin' in k['kernel'].lower():
        return 'null'
    return 'other'


def main():
    fetch, write, out = sys.argv[1:4]
    sub = sys.argv[4] if len(sys.argv) > 4 else 'rk_group_kernel'
    F, W = rows(fetch), rows(write)
    long_ms = max(r['ms'] for r in F + W if sub in r['kernel'])
    res = {'kernel': sub, 'fetch_correction': 'FETCH_SIZE x 2 (MI355X_MICROARCH.md, HBM [CDNA4])',
           'dispatches_fetch_pass': [], 'dispatches_write_pass': []}
    groups = {}
    for tag, lst in (('fetch', F), ('write', W)):
        for r in lst:
            c = classify(r, sub, long_ms)
            b = r['bytes'] * (2 if tag == 'fetch' else 1)
            res[f'dispatches_{tag}_pass'].append({'dispatch': r['dispatch'], 'class': c, 'kernel': r['kernel'][:70],
                                                  'ms': round(r['ms'], 4), 'bytes': b,
                                                  **({'fetch_size_raw_bytes': r['bytes']} if tag == 'fetch' else {})})
            groups.setdefault((c, tag), []).append(b)
    summ = {}
    for (c, tag), v in sorted(groups.items()):
        if c == 'other':
            continue
        summ[f'{c}_{tag}_bytes'] = {'launches': len(v), 'median': statistics.median(v), 'min': min(v), 'max': max(v),
                                    'all': v}
    res['summary'] = summ
    fl, wl = groups.get(('fine_long', 'fetch'), []), groups.get(('fine_long', 'write'), [])
    if fl and wl:
        res['bytes_per_launch'] = statistics.median(fl) + statistics.median(wl)
        res['bytes_per_launch_all'] = [a + b for a, b in zip(sorted(fl), sorted(wl))]
    fs, ws = groups.get(('fine_short', 'fetch'), []), groups.get(('fine_short', 'write'), [])
    if fs and ws:
        res['bytes_per_launch_short'] = statistics.median(fs) + statistics.median(ws)
    nf, nw = groups.get(('null', 'fetch'), []), groups.get(('null', 'write'), [])
    if nf and nw:
        res['null_kernel_bytes_median'] = statistics.median(nf) + statistics.median(nw)
    json.dump(res, open(out, 'w'), indent=1)
    print(json.dumps({k: v for k, v in res.items() if not k.startswith('dispatches')}, indent=1)[:3000])


if __name__ == '__main__':
    main()
