"""Per-launch HBM traffic of the fine kernel from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

FETCH_SIZE / WRITE_SIZE are in KiB.  MI355X_MICROARCH.md: on gfx950 FETCH_SIZE reads 1/2 of the
bytes of WIDE coalesced streaming reads; the fine kernel's reads are a few KiB of 8-byte loads,
so the raw value is reported (no x2), and the first (cold) launch is skipped.
Usage: python tools/pmc_traffic.py <fetch.csv> <write.csv> <out.json> [kernel-substring]
"""
import csv
import json
import sys


def values(path, sub):
    out = []
    for r in csv.DictReader(open(path)):
        if sub in r['Kernel_Name']:
            out.append(float(r['Counter_Value']) * 1024.0)
    return out


def main():
    fetch, write, out = sys.argv[1:4]
    sub = sys.argv[4] if len(sys.argv) > 4 else 'rk_group_kernel'
    f, w = values(fetch, sub), values(write, sub)
    f_warm = f[1:] if len(f) > 1 else f
    w_warm = w[1:] if len(w) > 1 else w
    res = {'kernel': sub, 'fetch_bytes_per_launch': sum(f_warm) / len(f_warm),
           'write_bytes_per_launch': sum(w_warm) / len(w_warm)}
    res['bytes_per_launch'] = res['fetch_bytes_per_launch'] + res['write_bytes_per_launch']
    res['launches'] = len(f)
    json.dump(res, open(out, 'w'), indent=1)
    print(res)


if __name__ == '__main__':
    main()
