"""Per-launch HBM traffic of the fine kernel from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

FETCH_SIZE / WRITE_SIZE are in KiB.  MI355X_MICROARCH.md: on gfx950 FETCH_SIZE reads 1/2 of the
bytes of WIDE coalesced streaming reads; the fine kernel's reads are a few KiB of 8-byte loads,
so the raw value is reported (no x2).  Per counter the MINIMUM over the launches is taken: the TCC
counters are device-wide over a multi-second launch, and one pass has seen 685 KiB written during a
launch whose own output is 3 KiB (another launch of the same pass: 3 KiB).
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
    res = {'kernel': sub, 'fetch_bytes_per_launch': min(f), 'write_bytes_per_launch': min(w),
           'fetch_bytes_all_launches': f, 'write_bytes_all_launches': w}
    res['bytes_per_launch'] = res['fetch_bytes_per_launch'] + res['write_bytes_per_launch']
    res['launches'] = len(f)
    json.dump(res, open(out, 'w'), indent=1)
    print(res)


if __name__ == '__main__':
    main()
